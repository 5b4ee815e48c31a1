"""Quaternion helpers (restated isaacgym.torch_utils) vs the scipy-pinned fixture."""
import numpy as np
import torch

from humanoid.utils.math import quat_rotate_inverse, quat_apply, get_euler_xyz_tensor
import envlogic_ref as E


def test_quat_helpers(golden):
    g = golden("quat.npz")
    q, v = torch.tensor(g["q"]), torch.tensor(g["v"])
    np.testing.assert_allclose(quat_rotate_inverse(q, v).numpy(), g["rot_inv"], atol=1e-12)
    np.testing.assert_allclose(quat_apply(q, v).numpy(), g["apply"], atol=1e-12)
    np.testing.assert_allclose(get_euler_xyz_tensor(q.float()).numpy(), g["euler"], atol=1e-6)
    np.testing.assert_allclose(E.quat_rotate_inverse(g["q"], g["v"]), g["rot_inv"], atol=1e-5)
    np.testing.assert_allclose(E.euler_xyz(g["q"]), g["euler"], atol=2e-6)
