"""Generate golden input/output vectors from the REFERENCE implementation.

Runs only in the build container (needs /root/reference, read-only).  The outputs are small .npz
fixtures committed under tests/golden/; the GPU box and the test-suite never read the reference.

Recipe:
  * PPO / RolloutStorage / ActorCritic: loaded by file path as a synthetic package 'refppo'
    (humanoid/algo/ppo/{actor_critic,rollout_storage,ppo}.py).
  * Env arithmetic: humanoid/envs/custom/humanoid_env.py imported with stub modules for
    isaacgym (gymapi, gymutil, gymtorch, terrain_utils, torch_utils), wandb and
    torch.utils.tensorboard; methods run on XBotLFreeEnv.__new__(XBotLFreeEnv) with synthetic
    state at the fork's native 18-DOF layout (its hard-coded +6 indices need 18 DOFs).
  * The isaacgym.torch_utils helpers used by the env are THIRD-PARTY (not in the reference tree);
    the stubs below restate Isaac Gym Preview 4's published definitions.  Values depending only
    on them are "parity unpinned" (see DESIGN.md).

Usage:  python tests/golden/gen_goldens.py   (writes tests/golden/*.npz)
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------------------------
# stubs
# ----------------------------------------------------------------------------------------------
def _torch_utils_module():
    tu = types.ModuleType("isaacgym.torch_utils")

    def quat_rotate_inverse(q, v):
        shape = q.shape
        q_w = q[:, -1]
        q_vec = q[:, :3]
        a = v * (2.0 * q_w ** 2 - 1.0).unsqueeze(-1)
        b = torch.cross(q_vec, v, dim=-1) * q_w.unsqueeze(-1) * 2.0
        c = q_vec * torch.bmm(q_vec.view(shape[0], 1, 3), v.view(shape[0], 3, 1)).squeeze(-1) * 2.0
        return a - b + c

    def quat_apply(a, b):
        shape = b.shape
        a = a.reshape(-1, 4)
        b = b.reshape(-1, 3)
        xyz = a[:, :3]
        t = xyz.cross(b, dim=-1) * 2
        return (b + a[:, 3:] * t + xyz.cross(t, dim=-1)).view(shape)

    def normalize(x, eps: float = 1e-9):
        return x / x.norm(p=2, dim=-1).clamp(min=eps, max=None).unsqueeze(-1)

    def copysign(a, b):
        a = torch.tensor(a, device=b.device, dtype=torch.float).repeat(b.shape[0])
        return torch.abs(a) * torch.sign(b)

    def get_euler_xyz(q):
        qx, qy, qz, qw = 0, 1, 2, 3
        sinr_cosp = 2.0 * (q[:, qw] * q[:, qx] + q[:, qy] * q[:, qz])
        cosr_cosp = q[:, qw] * q[:, qw] - q[:, qx] * q[:, qx] - q[:, qy] * q[:, qy] + q[:, qz] * q[:, qz]
        roll = torch.atan2(sinr_cosp, cosr_cosp)
        sinp = 2.0 * (q[:, qw] * q[:, qy] - q[:, qz] * q[:, qx])
        pitch = torch.where(torch.abs(sinp) >= 1, copysign(np.pi / 2.0, sinp), torch.asin(sinp))
        siny_cosp = 2.0 * (q[:, qw] * q[:, qz] + q[:, qx] * q[:, qy])
        cosy_cosp = q[:, qw] * q[:, qw] + q[:, qx] * q[:, qx] - q[:, qy] * q[:, qy] - q[:, qz] * q[:, qz]
        yaw = torch.atan2(siny_cosp, cosy_cosp)
        return roll % (2 * np.pi), pitch % (2 * np.pi), yaw % (2 * np.pi)

    def torch_rand_float(lower, upper, shape, device):
        return (upper - lower) * torch.rand(*shape, device=device) + lower

    def to_torch(x, dtype=torch.float, device="cuda:0", requires_grad=False):
        return torch.tensor(x, dtype=dtype, device=device, requires_grad=requires_grad)

    def get_axis_params(value, axis_idx, x_value=0.0, dtype=np.float64, n_dims=3):
        zs = np.zeros((n_dims,))
        assert axis_idx < n_dims
        zs[axis_idx] = 1.0
        params = np.where(zs == 1.0, value, zs)
        params[0] = x_value
        return list(params.astype(dtype))

    for f in (quat_rotate_inverse, quat_apply, normalize, copysign, get_euler_xyz, torch_rand_float,
              to_torch, get_axis_params):
        setattr(tu, f.__name__, f)
    tu.__all__ = [f.__name__ for f in (quat_rotate_inverse, quat_apply, normalize, copysign,
                                       get_euler_xyz, torch_rand_float, to_torch, get_axis_params)]
    tu.torch = torch
    tu.np = np
    return tu


def install_stubs():
    ig = types.ModuleType("isaacgym")
    ig.__path__ = []
    sys.modules["isaacgym"] = ig
    for sub in ("gymapi", "gymutil", "gymtorch", "terrain_utils"):
        m = types.ModuleType("isaacgym." + sub)
        sys.modules["isaacgym." + sub] = m
        setattr(ig, sub, m)
    tu = _torch_utils_module()
    sys.modules["isaacgym.torch_utils"] = tu
    ig.torch_utils = tu
    sys.modules["wandb"] = types.ModuleType("wandb")
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = object
    sys.modules["torch.utils.tensorboard"] = tb
    # skip package __init__ files that pull missing modules (humanoid/envs/__init__.py:39-43)
    sys.path.insert(0, REF)
    for pkg in ("humanoid.envs", "humanoid.utils", "humanoid.algo"):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(REF, *pkg.split("."))]
        sys.modules[pkg] = m


def load_ref_ppo():
    base = os.path.join(REF, "humanoid", "algo", "ppo")
    pkg = types.ModuleType("refppo")
    pkg.__path__ = [base]
    sys.modules["refppo"] = pkg
    mods = {}
    for name in ("actor_critic", "rollout_storage", "ppo"):
        spec = importlib.util.spec_from_file_location("refppo." + name, os.path.join(base, name + ".py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules["refppo." + name] = mod
        spec.loader.exec_module(mod)
        mods[name] = mod
    return mods


# ----------------------------------------------------------------------------------------------
# PPO goldens
# ----------------------------------------------------------------------------------------------
def gen_gae(mods):
    RS = mods["rollout_storage"].RolloutStorage
    out = {}
    for N in (4, 64):
        T = 24
        g = torch.Generator().manual_seed(100 + N)
        st = RS(N, T, [5], [7], [3], device="cpu")
        st.rewards[:] = torch.randn(T, N, 1, generator=g) * 0.3 + 0.1
        st.values[:] = torch.randn(T, N, 1, generator=g)
        st.dones[:] = (torch.rand(T, N, 1, generator=g) < 0.08).byte()
        last = torch.randn(N, 1, generator=g)
        out[f"N{N}_rewards"] = st.rewards[..., 0].numpy().copy()
        out[f"N{N}_values"] = st.values[..., 0].numpy().copy()
        out[f"N{N}_dones"] = st.dones[..., 0].numpy().copy()
        out[f"N{N}_last_values"] = last[:, 0].numpy().copy()
        st.compute_returns(last, 0.994, 0.9)
        out[f"N{N}_returns"] = st.returns[..., 0].numpy().copy()
        out[f"N{N}_advantages"] = st.advantages[..., 0].numpy().copy()
    np.savez_compressed(os.path.join(OUT, "gae.npz"), **out)


SMALL = dict(num_actor_obs=141, num_critic_obs=73, num_actions=12, actor_hidden_dims=[64, 32, 16],
             critic_hidden_dims=[48, 32, 16], base_lin_vel_hidden_dims=[24, 24], init_noise_std=1.0)


def sd_to_np(sd, prefix):
    return {prefix + k: v.detach().numpy().copy() for k, v in sd.items()}


def gen_actor_critic(mods):
    AC = mods["actor_critic"].ActorCritic
    torch.manual_seed(7)
    ac = AC(**SMALL)
    g = torch.Generator().manual_seed(8)
    obs = torch.randn(8, 141, generator=g)
    cobs = torch.randn(8, 73, generator=g)
    acts = torch.randn(8, 12, generator=g)
    with torch.no_grad():
        ac.std[:] = torch.linspace(0.5, 1.5, 12)
        mean = ac.act_inference(obs)
        ac.update_distribution(obs)
        logp = ac.get_actions_log_prob(acts)
        ent = ac.entropy
        val = ac.evaluate(cobs)
        lv = ac.base_get_lin_vel(obs)
        std = ac.action_std
    out = dict(obs=obs.numpy(), critic_obs=cobs.numpy(), actions=acts.numpy(), mean=mean.numpy(),
               log_prob=logp.numpy(), entropy=ent.numpy(), value=val.numpy(), lin_vel=lv.numpy(),
               action_std=std.numpy())
    out.update(sd_to_np(ac.state_dict(), "sd/"))
    np.savez_compressed(os.path.join(OUT, "actor_critic.npz"), **out)


def gen_ppo_update(mods):
    AC = mods["actor_critic"].ActorCritic
    PPO = mods["ppo"].PPO
    torch.manual_seed(11)
    ac = AC(**SMALL)
    ppo = PPO(ac, num_learning_epochs=2, num_mini_batches=4, clip_param=0.2, gamma=0.994, lam=0.9,
              value_loss_coef=1.0, entropy_coef=0.001, learning_rate=1e-5, max_grad_norm=1.0,
              use_clipped_value_loss=True, schedule="adaptive", desired_kl=0.01, device="cpu")
    N, T = 8, 24
    ppo.init_storage(N, T, [141], [73], [12])
    init_sd = {k: v.clone() for k, v in ac.state_dict().items()}
    g = torch.Generator().manual_seed(12)
    rec = {k: [] for k in ("obs", "critic_obs", "rewards", "dones", "time_outs")}
    with torch.inference_mode():
        for t in range(T):
            obs = torch.randn(N, 141, generator=g)
            cobs = torch.randn(N, 73, generator=g)
            ppo.act(obs, cobs)
            rew = torch.rand(N, generator=g)
            dones = torch.rand(N, generator=g) < 0.1
            tos = dones & (torch.rand(N, generator=g) < 0.5)
            ppo.process_env_step(rew, dones, {"time_outs": tos})
            for k, v in zip(rec, (obs, cobs, rew, dones, tos)):
                rec[k].append(v.clone())
        last_cobs = torch.randn(N, 73, generator=g)
        ppo.compute_returns(last_cobs)
    st = ppo.storage
    out = dict(last_critic_obs=last_cobs.numpy())
    for k in ("observations", "privileged_observations", "actions", "rewards", "dones", "values",
              "actions_log_prob", "mu", "sigma", "returns", "advantages"):
        out["st/" + k] = getattr(st, k).numpy().copy()
    out.update(sd_to_np(init_sd, "init/"))
    torch.manual_seed(1234)
    vloss, sloss, sym, lvloss = ppo.update()
    out.update(value_loss=np.float64(vloss), surrogate_loss=np.float64(sloss),
               lin_vel_loss=np.float64(lvloss), learning_rate=np.float64(ppo.learning_rate))
    out.update(sd_to_np(ac.state_dict(), "final/"))
    np.savez_compressed(os.path.join(OUT, "ppo_update.npz"), **out)


# ----------------------------------------------------------------------------------------------
# env goldens (18-DOF fork layout)
# ----------------------------------------------------------------------------------------------
def make_env_state(E, he, N, seed):
    from humanoid.envs.custom.humanoid_config import XBotLCfg
    tu = sys.modules["isaacgym.torch_utils"]
    g = torch.Generator().manual_seed(seed)
    D, B = 18, 13

    def U(lo, hi, *shape):
        return (hi - lo) * torch.rand(*shape, generator=g) + lo

    cfg = XBotLCfg()
    E.cfg = cfg
    E.device = "cpu"
    E.num_envs = N
    E.num_actions = D
    E.num_dof = D
    E.dt = cfg.control.decimation * 0.001
    E.obs_scales = cfg.normalization.obs_scales
    E.max_episode_length = np.ceil(cfg.env.episode_length_s / E.dt)
    E.feet_indices = torch.tensor([6, 12])
    E.knee_indices = torch.tensor([4, 10])
    E.penalised_contact_indices = torch.tensor([0])
    E.termination_contact_indices = torch.tensor([0])
    E.episode_length_buf = torch.randint(0, 2600, (N,), generator=g)
    E.dof_pos = U(-0.6, 0.6, N, D)
    E.dof_vel = U(-4, 4, N, D)
    E.default_dof_pos = U(-0.3, 0.3, 1, D)
    E.default_joint_pd_target = E.default_dof_pos.clone()
    E.actions = U(-3, 3, N, D)
    E.last_actions = U(-3, 3, N, D)
    E.last_last_actions = U(-3, 3, N, D)
    E.torques = U(-150, 150, N, D)
    E.last_dof_vel = U(-4, 4, N, D)
    q = torch.cat([U(-0.15, 0.15, N, 3), torch.ones(N, 1)], dim=1)
    q = q / q.norm(dim=1, keepdim=True)
    E.root_states = torch.cat([U(-2, 2, N, 2), U(0.75, 1.05, N, 1), q, U(-1, 1, N, 6)], dim=1)
    E.last_root_vel = E.root_states[:, 7:13] + U(-0.3, 0.3, N, 6)
    E.base_quat = E.root_states[:, 3:7]
    E.base_lin_vel = tu.quat_rotate_inverse(E.base_quat, E.root_states[:, 7:10])
    E.base_ang_vel = tu.quat_rotate_inverse(E.base_quat, E.root_states[:, 10:13])
    E.gravity_vec = torch.tensor([[0.0, 0.0, -1.0]]).repeat(N, 1)
    E.projected_gravity = tu.quat_rotate_inverse(E.base_quat, E.gravity_vec)
    E.base_euler_xyz = he.get_euler_xyz_tensor(E.base_quat)
    rs = torch.zeros(N, B, 13)
    rs[:, :, 0:2] = U(-1, 1, N, B, 2)
    rs[:, :, 2] = U(0.0, 0.16, N, B)
    rs[:, :, 3:7] = q[:, None, :]
    rs[:, :, 7:13] = U(-2, 2, N, B, 6)
    rs[:, 12, 0:2] = rs[:, 6, 0:2] + U(-0.6, 0.6, N, 2)
    rs[:, 10, 0:2] = rs[:, 4, 0:2] + U(-0.35, 0.35, N, 2)
    E.rigid_state = rs
    cf = torch.zeros(N, B, 3)
    cf[:, :, :] = U(-3, 3, N, B, 3)
    cf[:, :, 2] = U(0, 12, N, B)
    cf[:, 0, :] *= (torch.rand(N, 1, generator=g) < 0.3).float() * 2.0   # base contact for some
    big = torch.rand(N, generator=g) < 0.25
    cf[big, 6, 2] = U(650, 1300, int(big.sum()))
    E.contact_forces = cf
    cmd = torch.cat([U(-0.3, 0.6, N, 1), U(-0.3, 0.3, N, 1), U(-0.3, 0.3, N, 1), U(-3.14, 3.14, N, 1)], 1)
    cmd[::5, 0] = 0.05
    E.commands = cmd
    E.commands_scale = torch.tensor([E.obs_scales.lin_vel, E.obs_scales.lin_vel, E.obs_scales.ang_vel])
    E.feet_air_time = U(0, 0.6, N, 2) * (torch.rand(N, 2, generator=g) < 0.7).float()
    E.last_contacts = torch.rand(N, 2, generator=g) < 0.5
    E.feet_height = U(0, 0.13, N, 2)
    E.last_feet_z = U(0.0, 0.1, N, 2)
    E.rand_push_force = U(-0.2, 0.2, N, 3)
    E.rand_push_torque = U(-0.4, 0.4, N, 3)
    E.env_frictions = U(0.1, 2.0, N, 1)
    E.body_mass = U(25, 35, N, 1)
    return g


def gen_env(he):
    from collections import deque
    XB = he.XBotLFreeEnv
    out = {}
    N = 32
    E = XB.__new__(XB)
    g = make_env_state(E, he, N, seed=21)
    E.reward_scales = he.class_to_dict(E.cfg.rewards.scales)
    E.rew_buf = torch.zeros(N)
    E._prepare_reward_function()
    names = list(E.reward_names)
    for k in ("dof_pos", "dof_vel", "default_dof_pos", "actions", "last_actions", "last_last_actions",
              "torques", "last_dof_vel", "root_states", "last_root_vel", "rigid_state", "contact_forces",
              "commands", "feet_air_time", "last_contacts", "feet_height", "last_feet_z",
              "rand_push_force", "rand_push_torque", "env_frictions", "body_mass", "episode_length_buf",
              "base_lin_vel", "base_ang_vel", "projected_gravity", "base_euler_xyz"):
        v = getattr(E, k)
        out["in/" + k] = v.numpy().copy() if torch.is_tensor(v) else np.asarray(v)
    out["reward_names"] = np.array(names)
    out["reward_scales"] = np.array([E.reward_scales[n] for n in names], dtype=np.float64)
    # torques (PD) with p/d gains per 18-dof fork config
    E.p_gains = torch.rand(N, 18, generator=g) * 300
    E.d_gains = torch.rand(N, 18, generator=g) * 10
    E.torque_limits = torch.rand(18, generator=g) * 150 + 20
    acts = (torch.rand(N, 18, generator=g) - 0.5) * 8
    out["pd/p_gains"] = E.p_gains.numpy().copy()
    out["pd/d_gains"] = E.d_gains.numpy().copy()
    out["pd/torque_limits"] = E.torque_limits.numpy().copy()
    out["pd/actions"] = acts.numpy().copy()
    out["pd/torques"] = E._compute_torques(acts).numpy().copy()
    # phase / gait / ref
    out["phase"] = E._get_phase().numpy().copy()
    out["stance_mask"] = E._get_gait_phase().numpy().copy()
    E.compute_ref_state()
    out["ref_dof_pos"] = E.ref_dof_pos.numpy().copy()
    out["ref_action"] = E.ref_action.numpy().copy()
    out["noise_vec"] = E._get_noise_scale_vec(E.cfg).numpy().copy()
    # termination
    E.check_termination()
    out["reset_buf"] = E.reset_buf.numpy().copy()
    out["time_out_buf"] = E.time_out_buf.numpy().copy()
    # rewards, term by term (wrapped to record the exact values compute_reward consumes)
    terms = {}

    def wrap(n, f):
        def w():
            r = f()
            terms[n] = r.detach().clone()
            return r
        return w

    E.reward_functions = [wrap(n, f) for n, f in zip(names, E.reward_functions)]
    E.compute_reward()
    for n in names:
        out["term/" + n] = terms[n].float().numpy().copy()
        out["sum/" + n] = E.episode_sums[n].numpy().copy()
    out["rew_buf"] = E.rew_buf.numpy().copy()
    for k in ("feet_air_time", "last_contacts", "feet_height", "last_feet_z"):
        v = getattr(E, k)
        out["post/" + k] = v.numpy().copy() if torch.is_tensor(v) else np.asarray(v)
    # observations, 3 consecutive calls with changing state (history stacking)
    E.add_noise = False
    E.obs_history = deque(maxlen=E.cfg.env.frame_stack)
    E.critic_history = deque(maxlen=E.cfg.env.c_frame_stack)
    for _ in range(E.cfg.env.frame_stack):
        E.obs_history.append(torch.zeros(N, E.cfg.env.num_single_obs))
    for _ in range(E.cfg.env.c_frame_stack):
        E.critic_history.append(torch.zeros(N, E.cfg.env.single_num_privileged_obs))
    for it in range(3):
        E.episode_length_buf = E.episode_length_buf + 1
        E.dof_pos = E.dof_pos + 0.05 * torch.randn(N, 18, generator=g)
        E.actions = E.actions + 0.1 * torch.randn(N, 18, generator=g)
        out[f"obs{it}/dof_pos"] = E.dof_pos.numpy().copy()
        out[f"obs{it}/actions"] = E.actions.numpy().copy()
        out[f"obs{it}/episode_length_buf"] = E.episode_length_buf.numpy().copy()
        E.compute_observations()
        out[f"obs{it}/obs_buf"] = E.obs_buf.numpy().copy()
        out[f"obs{it}/privileged_obs_buf"] = E.privileged_obs_buf.numpy().copy()
    np.savez_compressed(os.path.join(OUT, "env18.npz"), **out)


def gen_math(he):
    """Quaternion helpers vs scipy (pins the torch_utils restatement)."""
    from scipy.spatial.transform import Rotation
    tu = sys.modules["isaacgym.torch_utils"]
    rng = np.random.default_rng(3)
    q = rng.normal(size=(64, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    v = rng.normal(size=(64, 3))
    qt, vt = torch.tensor(q, dtype=torch.float64), torch.tensor(v, dtype=torch.float64)
    R = Rotation.from_quat(q)  # scipy uses xyzw like Isaac Gym
    rot_inv = tu.quat_rotate_inverse(qt, vt).numpy()
    assert np.allclose(rot_inv, R.inv().apply(v), atol=1e-10)
    app = tu.quat_apply(qt, vt).numpy()
    assert np.allclose(app, R.apply(v), atol=1e-10)
    eul = he.get_euler_xyz_tensor(qt.float()).numpy()
    sc = R.as_euler("xyz")  # extrinsic xyz == roll/pitch/yaw
    d = np.angle(np.exp(1j * (eul - sc)))
    assert np.abs(d).max() < 1e-4, np.abs(d).max()
    np.savez_compressed(os.path.join(OUT, "quat.npz"), q=q, v=v, rot_inv=rot_inv, apply=app, euler=eul)


def main():
    torch.set_num_threads(1)
    mods = load_ref_ppo()
    gen_gae(mods)
    gen_actor_critic(mods)
    gen_ppo_update(mods)
    install_stubs()
    from humanoid.envs.custom import humanoid_env as he
    gen_env(he)
    gen_math(he)
    print("goldens written to", OUT)


if __name__ == "__main__":
    main()
