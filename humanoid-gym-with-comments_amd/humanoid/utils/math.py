"""Quaternion / angle helpers (reference humanoid/utils/math.py:39-57 and the
isaacgym.torch_utils functions the env uses via `from isaacgym.torch_utils import *`,
humanoid_env.py:35).  The torch_utils restatements follow Isaac Gym Preview 4's published
definitions (third-party, not in the reference tree): parity for them is pinned only by the
scipy check in tests/golden/quat.npz."""
import numpy as np
import torch

__all__ = ["quat_apply_yaw", "wrap_to_pi", "torch_rand_sqrt_float", "quat_rotate_inverse", "quat_apply",
           "normalize", "get_euler_xyz", "get_euler_xyz_tensor", "torch_rand_float", "to_torch",
           "get_axis_params", "copysign"]


def normalize(x, eps: float = 1e-9):
    return x / x.norm(p=2, dim=-1).clamp(min=eps).unsqueeze(-1)


def quat_apply(a, b):
    shape = b.shape
    a = a.reshape(-1, 4)
    b = b.reshape(-1, 3)
    xyz = a[:, :3]
    t = torch.cross(xyz, b, dim=-1) * 2
    return (b + a[:, 3:] * t + torch.cross(xyz, t, dim=-1)).view(shape)


def quat_rotate_inverse(q, v):
    qw = q[:, -1:]
    qv = q[:, :3]
    return (v * (2.0 * qw ** 2 - 1.0) - torch.cross(qv, v, dim=-1) * qw * 2.0
            + qv * (qv * v).sum(dim=-1, keepdim=True) * 2.0)


def copysign(a, b):
    return torch.abs(torch.full_like(b, a)) * torch.sign(b)


def get_euler_xyz(q):
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    roll = torch.atan2(2.0 * (w * x + y * z), w * w - x * x - y * y + z * z)
    sinp = 2.0 * (w * y - z * x)
    pitch = torch.where(torch.abs(sinp) >= 1, copysign(np.pi / 2.0, sinp), torch.asin(sinp.clamp(-1, 1)))
    yaw = torch.atan2(2.0 * (w * z + x * y), w * w + x * x - y * y - z * z)
    return roll % (2 * np.pi), pitch % (2 * np.pi), yaw % (2 * np.pi)


def get_euler_xyz_tensor(quat):
    """Euler xyz wrapped to (-pi, pi] (humanoid_env.py:51-56)."""
    e = torch.stack(get_euler_xyz(quat), dim=1)
    e[e > np.pi] -= 2 * np.pi
    return e


def torch_rand_float(lower, upper, shape, device):
    return (upper - lower) * torch.rand(*shape, device=device) + lower


def to_torch(x, dtype=torch.float, device="cuda:0", requires_grad=False):
    return torch.tensor(x, dtype=dtype, device=device, requires_grad=requires_grad)


def get_axis_params(value, axis_idx, x_value=0.0, dtype=np.float64, n_dims=3):
    p = np.zeros(n_dims, dtype=dtype)
    p[axis_idx] = value
    p[0] = x_value
    return list(p)


def quat_apply_yaw(quat, vec):
    q = quat.clone().view(-1, 4)
    q[:, :2] = 0.0
    return quat_apply(normalize(q), vec)


def wrap_to_pi(angles):
    angles %= 2 * np.pi
    angles -= 2 * np.pi * (angles > np.pi)
    return angles


def torch_rand_sqrt_float(lower, upper, shape, device):
    r = 2 * torch.rand(*shape, device=device) - 1
    r = torch.where(r < 0.0, -torch.sqrt(-r), torch.sqrt(r))
    return (upper - lower) * (r + 1.0) / 2.0 + lower
