"""XBotLFreeEnv on hg_sim: the reference env API (humanoid/envs/custom/humanoid_env.py:63-1437)
with the physics and all per-step env arithmetic running in HIP kernels.

Python keeps what the reference does once (config parsing, model load, domain-randomisation
draws at creation, reward-function bookkeeping) and the host-side step counter; every per-step
operation is one hg_step (action preprocessing + 10 physics substeps) and one hg_post
(derived state, commands, push, termination, 22 rewards, masked reset, observations, history
stacking) launched on the current stream — no host synchronisation.

Tensor attributes (root_states, dof_pos, contact_forces, rigid_state, commands, rew_buf, ...)
are zero-copy views into the simulator's SoA arena, so they read and write like the reference's
gymtorch-wrapped tensors (``root_states[:, 3:7]``, ``dof_pos[env_ids] = ...``).
"""
import ctypes

import numpy as np
import torch

from humanoid import _native as N
from humanoid.envs.base.base_task import BaseTask
from humanoid.utils.helpers import class_to_dict
from humanoid.utils.math import quat_rotate_inverse, get_euler_xyz_tensor  # noqa: F401
from .humanoid_config import XBotLCfg  # noqa: F401

REWARD_NAMES = [
    "action_smoothness", "base_acc", "base_height", "collision", "default_joint_pos", "dof_acc", "dof_vel",
    "feet_air_time", "feet_clearance", "feet_contact_forces", "feet_contact_number", "feet_distance",
    "foot_slip", "joint_pos", "knee_distance", "low_speed", "orientation", "torques", "track_vel_hard",
    "tracking_ang_vel", "tracking_lin_vel", "vel_mismatch_exp",
]
assert REWARD_NAMES == sorted(REWARD_NAMES)

_TORCH_DTYPES = {0: torch.float32, 1: torch.int64, 2: torch.uint8, 3: torch.int32}


def build_hg_cfg(cfg, num_envs, sim_dt, seed, model_js, heightfield=None, hf_shape=(0, 0), terrain_origins=None,
                 terrain_shape=(0, 0)):
    """XBotLCfg -> hg_cfg (include/hgsim.h).  Returns (hg_cfg, aux dict)."""
    c = N.HgCfg()
    c.num_envs = num_envs
    c.decimation = cfg.control.decimation
    it = getattr(cfg.sim.hg, "pgs_iterations", None)
    if it is None:
        px = cfg.sim.physx
        it = int(px.num_position_iterations) + int(getattr(px, "num_velocity_iterations", 0))
    c.pgs_iterations = max(1, int(it))
    c.fix_base_link = int(cfg.asset.fix_base_link)
    c.sim_dt = sim_dt
    c.gravity_z = cfg.sim.gravity[2]
    c.contact_offset = cfg.sim.physx.contact_offset
    c.max_depenetration_vel = cfg.sim.physx.max_depenetration_velocity
    c.baumgarte = cfg.sim.hg.baumgarte
    c.ground_friction = cfg.terrain.static_friction
    c.action_scale = cfg.control.action_scale
    c.clip_actions = cfg.normalization.clip_actions
    c.dynamic_randomization = cfg.domain_rand.dynamic_randomization
    bodies, dofs, effort, limits, velocity = N.model_names(model_js)
    kp, kd, tl, dd = [], [], [], []
    for j, name in enumerate(dofs):
        # substring match, last match wins (humanoid_env.py:285-297)
        p = d = 0.0
        for key in cfg.control.stiffness:
            if key in name:
                p, d = cfg.control.stiffness[key], cfg.control.damping[key]
        kp.append(p)
        kd.append(d)
        tl.append(effort[j] * cfg.safety.torque_limit)
        dd.append(cfg.init_state.default_joint_angles.get(name, 0.0))
    for j in range(12):
        c.kp[j], c.kd[j], c.torque_limit[j], c.default_dof_pos[j] = kp[j], kd[j], tl[j], dd[j]
    if heightfield is not None:
        c.terrain_type = 1
        c.hf_rows, c.hf_cols = hf_shape
        c.hf_horizontal_scale = cfg.terrain.horizontal_scale
        c.hf_vertical_scale = cfg.terrain.vertical_scale
        c.hf_border = cfg.terrain.border_size
        c.heightfield = heightfield
    dt = cfg.control.decimation * sim_dt
    c.frame_stack = cfg.env.frame_stack
    c.c_frame_stack = cfg.env.c_frame_stack
    c.max_episode_length = int(np.ceil(cfg.env.episode_length_s / dt))
    c.resample_interval = int(cfg.commands.resampling_time / dt)
    c.push_interval = int(np.ceil(cfg.domain_rand.push_interval_s / dt))
    c.push_robots = int(cfg.domain_rand.push_robots)
    c.add_noise = int(cfg.noise.add_noise)
    c.heading_command = int(cfg.commands.heading_command)
    c.only_positive_rewards = int(cfg.rewards.only_positive_rewards)
    c.dt = dt
    r = cfg.rewards
    c.cycle_time, c.target_joint_pos_scale, c.target_feet_height = r.cycle_time, r.target_joint_pos_scale, r.target_feet_height
    c.base_height_target, c.min_dist, c.max_dist = r.base_height_target, r.min_dist, r.max_dist
    c.tracking_sigma, c.max_contact_force = r.tracking_sigma, r.max_contact_force
    c.max_push_vel_xy, c.max_push_ang_vel = cfg.domain_rand.max_push_vel_xy, cfg.domain_rand.max_push_ang_vel
    rg = cfg.commands.ranges
    for dst, src in ((c.cmd_lin_x, rg.lin_vel_x), (c.cmd_lin_y, rg.lin_vel_y), (c.cmd_ang_yaw, rg.ang_vel_yaw),
                     (c.cmd_heading, rg.heading)):
        dst[0], dst[1] = src
    ns, os_ = cfg.noise.noise_scales, cfg.normalization.obs_scales
    c.noise_level, c.noise_dof_pos, c.noise_dof_vel = cfg.noise.noise_level, ns.dof_pos, ns.dof_vel
    c.noise_ang_vel, c.noise_quat = ns.ang_vel, ns.quat
    c.obs_lin_vel, c.obs_ang_vel, c.obs_dof_pos, c.obs_dof_vel, c.obs_quat = (os_.lin_vel, os_.ang_vel, os_.dof_pos,
                                                                              os_.dof_vel, os_.quat)
    c.clip_observations = cfg.normalization.clip_observations
    st = cfg.init_state
    for i in range(3):
        c.init_pos[i], c.init_lin_vel[i], c.init_ang_vel[i] = st.pos[i], st.lin_vel[i], st.ang_vel[i]
    for i in range(4):
        c.init_rot[i] = st.rot[i]
    scales = class_to_dict(cfg.rewards.scales)
    for k, name in enumerate(REWARD_NAMES):
        c.reward_scale[k] = scales.get(name, 0.0) * dt
    feet = [i for i, b in enumerate(bodies) if cfg.asset.foot_name in b]
    knees = [i for i, b in enumerate(bodies) if cfg.asset.knee_name in b]
    c.feet_body[0], c.feet_body[1] = feet
    c.knee_body[0], c.knee_body[1] = knees
    # 12-DOF index maps: ref-state pitch/knee/ankle-pitch, default-pose yaw/roll
    idx = {n: i for i, n in enumerate(dofs)}
    for k, n in enumerate(["left_leg_pitch_joint", "left_knee_joint", "left_ankle_pitch_joint",
                           "right_leg_pitch_joint", "right_knee_joint", "right_ankle_pitch_joint"]):
        c.ref_idx[k] = idx[n]
    for k, n in enumerate(["left_leg_roll_joint", "left_leg_yaw_joint", "right_leg_roll_joint", "right_leg_yaw_joint"]):
        c.yaw_roll_idx[k] = idx[n]
    c.seed = seed & 0xFFFFFFFFFFFFFFFF
    c.env_offset = int(getattr(cfg.env, "env_offset", 0))
    c.max_episode_length_s = cfg.env.episode_length_s
    c.terrain_env_length = cfg.terrain.terrain_length
    if terrain_origins is not None and cfg.terrain.curriculum:
        c.curriculum = 1
        c.terrain_rows, c.terrain_cols = terrain_shape
        c.terrain_origins = terrain_origins
    aux = dict(feet=feet, knees=knees, dof_names=dofs, body_names=bodies, kp=kp, kd=kd, torque_limits=tl,
               default_dof_pos=dd, limits=limits, velocity=velocity, scales=scales)
    return c, aux



def _live(view):
    """Tag a window view handed out in place of a copy (stable_observations False): the next step
    rewrites it, so a consumer that keeps it past env.step must copy it (PPO.act does)."""
    view.hg_live_view = True
    return view

class XBotLFreeEnv(BaseTask):
    """Drop-in for the reference XBotLFreeEnv (humanoid_env.py:63)."""

    def __init__(self, cfg, sim_params, physics_engine, sim_device, headless):
        self.cfg = cfg
        self.sim_params = sim_params
        self.height_samples = None
        self.debug_viz = False
        self.init_done = False
        self.kernel_timer = None  # optional: object with start(name)/stop(name) (bench.py HIP-event timer)
        self._parse_cfg(self.cfg)
        super().__init__(cfg, sim_params, physics_engine, sim_device, headless)
        self._init_buffers()
        self._prepare_reward_function()
        # step() / get_observations() hand out tensors that stay valid across later steps, as the
        # reference's (its compute_observations allocates a new obs_buf per step,
        # humanoid_env.py:880-887): a copy of the current window stack.  OnPolicyRunner turns this
        # off — its PPO copies the stack into the rollout storage before the next step — and then
        # the returned tensors are the live strided window views, valid until the next step()
        # (a reset zeroes that env's older frames in place).
        self.stable_observations = True
        self.init_done = True
        # reset_idx(all) + compute_observations() (humanoid_env.py:176-178)
        self._launch_reset(None)

    # ------------------------------------------------------------------ config
    def _parse_cfg(self, cfg):
        sim_dt = getattr(self.sim_params, "dt", None) or cfg.sim.dt
        self.sim_dt = sim_dt
        self.dt = cfg.control.decimation * sim_dt
        self.obs_scales = cfg.normalization.obs_scales
        self.reward_scales = class_to_dict(cfg.rewards.scales)
        self.command_ranges = class_to_dict(cfg.commands.ranges)
        if cfg.terrain.mesh_type not in ["heightfield", "trimesh"]:
            cfg.terrain.curriculum = False
        self.max_episode_length_s = cfg.env.episode_length_s
        self.max_episode_length = np.ceil(self.max_episode_length_s / self.dt)
        cfg.domain_rand.push_interval = np.ceil(cfg.domain_rand.push_interval_s / self.dt)

    def _prepare_reward_function(self):
        """Drop zero scales, multiply by dt; names in alphabetical order (humanoid_env.py:201-226)."""
        for key in list(self.reward_scales.keys()):
            if self.reward_scales[key] == 0:
                self.reward_scales.pop(key)
            else:
                self.reward_scales[key] *= self.dt
        self.reward_names = [n for n in self.reward_scales if n != "termination"]
        unknown = [n for n in self.reward_names if n not in REWARD_NAMES]
        if unknown:
            raise ValueError(f"reward terms without a HIP implementation: {unknown}")
        self.episode_sums = {name: self._sums[REWARD_NAMES.index(name)] for name in self.reward_names}

    # ------------------------------------------------------------------ creation
    def create_sim(self):
        """Model load, terrain, domain randomisation and the hg_sim handle
        (replaces create_sim/_create_envs, humanoid_env.py:333-524)."""
        self.up_axis_idx = 2
        self.hg = N.lib()
        hgc = self.cfg.sim.hg
        model, js = N.load_model(armature=hgc.armature, joint_friction=getattr(hgc, "joint_friction", True),
                                 self_collisions=self.cfg.asset.self_collisions == 0)
        self._model, self._model_js = model, js
        mesh = self.cfg.terrain.mesh_type
        hf_ptr, hf_shape = None, (0, 0)
        self.custom_origins = False
        if mesh == "plane":
            pass
        elif mesh in ("heightfield", "trimesh"):
            # 'trimesh' collides against the same triangulated heightfield (cells split along the
            # (i,j)-(i+1,j+1) diagonal, the tessellation of convert_heightfield_to_trimesh).
            # Every data-parallel rank must build the identical map: the generator runs on a
            # private numpy stream seeded by terrain.seed (default: the run seed), then the global
            # numpy state is restored.
            from humanoid.utils.terrain import HumanoidTerrain
            tseed = getattr(self.cfg.terrain, "seed", None)
            tseed = int(getattr(self.cfg, "seed", 5)) if tseed is None else int(tseed)
            saved = np.random.get_state()
            np.random.seed(tseed)
            try:
                self.terrain = HumanoidTerrain(self.cfg.terrain, self.num_envs)
            finally:
                np.random.set_state(saved)
            self.height_samples = torch.tensor(self.terrain.heightsamples, dtype=torch.int16, device=self.device)
            hf_ptr, hf_shape = self.height_samples.data_ptr(), tuple(self.height_samples.shape)
            self.custom_origins = True
        elif mesh is not None:
            raise ValueError("Terrain mesh type not recognised. Allowed types are [None, plane, heightfield, trimesh]")
        seed = int(getattr(self.cfg, "seed", 5))
        to_ptr, to_shape = None, (0, 0)
        if self.custom_origins:
            self.terrain_origins = torch.from_numpy(self.terrain.env_origins).to(self.device).to(torch.float).contiguous()
            to_ptr, to_shape = self.terrain_origins.data_ptr(), tuple(self.terrain_origins.shape[:2])
        self._hgcfg, self._aux = build_hg_cfg(self.cfg, self.num_envs, self.sim_dt, seed, js, hf_ptr, hf_shape,
                                              to_ptr, to_shape)
        nbytes = self.hg.hg_arena_bytes(ctypes.byref(self._hgcfg))
        self._arena = torch.empty(nbytes + 256, dtype=torch.uint8, device=self.device)
        off = (-self._arena.data_ptr()) % 256
        self._arena_base = self._arena[off:off + nbytes]
        handle = ctypes.c_void_p()
        N.check(self.hg.hg_create(ctypes.byref(self._hgcfg), ctypes.byref(model),
                                  ctypes.c_void_p(self._arena_base.data_ptr()), ctypes.c_size_t(nbytes),
                                  ctypes.byref(handle)))
        self.sim = handle
        self.num_dof = self.num_dofs = 12
        self.num_bodies = len(self._aux["body_names"])
        self.dof_names = self._aux["dof_names"]
        self.feet_indices = torch.tensor(self._aux["feet"], dtype=torch.long, device=self.device)
        self.knee_indices = torch.tensor(self._aux["knees"], dtype=torch.long, device=self.device)
        self.penalised_contact_indices = torch.tensor([0], dtype=torch.long, device=self.device)
        self.termination_contact_indices = torch.tensor([0], dtype=torch.long, device=self.device)
        self._wrap_all()
        self._get_env_origins()
        self._randomize_props()

    def _view(self, tid):
        d = N.HgDesc()
        N.check(self.hg.hg_tensor(self.sim, tid, ctypes.byref(d)), self.sim)
        dt = _TORCH_DTYPES[d.dtype]
        es = torch.empty((), dtype=dt).element_size()
        assert d.offset_bytes % es == 0
        shape = [d.shape[i] for i in range(d.ndim)]
        strides = [d.strides[i] for i in range(d.ndim)]
        return self._arena_base.view(dt).as_strided(shape, strides, d.offset_bytes // es)

    def _wrap_all(self):
        T = N.T
        self.root_states = self._view(T["ROOT_STATE"])
        self.dof_pos = self._view(T["DOF_POS"])
        self.dof_vel = self._view(T["DOF_VEL"])
        self.contact_forces = self._view(T["CONTACT_FORCES"])
        self.rigid_state = self._view(T["RIGID_STATE"])
        self.torques = self._view(T["TORQUES"])
        self.actions = self._view(T["ACTIONS"])
        self.last_actions = self._view(T["LAST_ACTIONS"])
        self.last_last_actions = self._view(T["LAST_LAST_ACTIONS"])
        self.last_dof_vel = self._view(T["LAST_DOF_VEL"])
        self.last_root_vel = self._view(T["LAST_ROOT_VEL"])
        self.commands = self._view(T["COMMANDS"])
        # observation histories: one sliding window per env row (HG_T_OBS_BUF / HG_T_PRIV_BUF); the
        # stacks are the [N, F * width] column slices at the sim's head slot (hg_obs_head), one
        # fixed strided view per head position (no tensor indexing per access)
        self._obs_win = self._view(T["OBS_BUF"])
        self._priv_win = self._view(T["PRIV_BUF"])
        hw = int(self.hg.hg_obs_window_advance(self.sim))
        fo, fp = int(self.cfg.env.frame_stack), int(self.cfg.env.c_frame_stack)
        wo, wp = self._obs_win.shape[1] // (fo - 1 + hw), self._priv_win.shape[1] // (fp - 1 + hw)
        self._obs_views = tuple(self._obs_win[:, h * wo:(h + fo) * wo] for h in range(hw))
        self._priv_views = tuple(self._priv_win[:, h * wp:(h + fp) * wp] for h in range(hw))
        self.rew_buf = self._view(T["REW_BUF"])
        self._reset_u8 = self._view(T["RESET_BUF"])
        self._timeout_u8 = self._view(T["TIME_OUT_BUF"])
        self.reset_buf = self._reset_u8.view(torch.bool)
        self.time_out_buf = self._timeout_u8.view(torch.bool)
        self._ep_len = self._view(T["EPISODE_LENGTH"])
        self._sums = self._view(T["EPISODE_SUMS"])
        self.feet_air_time = self._view(T["FEET_AIR_TIME"])
        self.last_contacts = self._view(T["LAST_CONTACTS"]).view(torch.bool)
        self.feet_height = self._view(T["FEET_HEIGHT"])
        self.last_feet_z = self._view(T["LAST_FEET_Z"])
        self.env_frictions = self._view(T["ENV_FRICTION"]).unsqueeze(1)
        self.body_mass = self._view(T["BODY_MASS"]).unsqueeze(1)
        self.rand_push_force = self._view(T["PUSH_FORCE"])
        self.rand_push_torque = self._view(T["PUSH_TORQUE"])
        self.base_lin_vel = self._view(T["BASE_LIN_VEL"])
        self.base_ang_vel = self._view(T["BASE_ANG_VEL"])
        self.projected_gravity = self._view(T["PROJ_GRAVITY"])
        self.base_euler_xyz = self._view(T["BASE_EULER"])
        self.ref_dof_pos = self._view(T["REF_DOF_POS"])
        self.env_origins = self._view(T["ENV_ORIGINS"])
        self._ep_stats = self._view(T["EP_STATS"])
        self._ep_ring = self._view(T["EP_STATS_RING"])
        self.nonfinite_count = self._view(T["NONFINITE"])
        # constraint rows / contact points the solver's row budget dropped, per env, summed over
        # substeps (diagnostic; 0 in normal operation)
        self.rows_dropped = self._view(T["ROWS_DROPPED"])

    def _global_ids(self):
        """(offset, total): this shard's envs are global ids [offset, offset + num_envs) of total."""
        off = int(getattr(self.cfg.env, "env_offset", 0))
        total = getattr(self.cfg.env, "num_envs_total", None)
        total = self.num_envs if total is None else int(total)
        if off < 0 or off + self.num_envs > total:
            raise ValueError(f"env shard [{off}, {off + self.num_envs}) outside num_envs_total={total}")
        return off, total

    def _creation_generator(self, stream):
        """Creation-time draws over ALL global envs from a private generator keyed by the run seed
        (the same on every rank), sliced to this shard; the global torch / numpy state is untouched."""
        g = torch.Generator()
        g.manual_seed((int(getattr(self.cfg, "seed", 5)) * 1000003 + stream) & 0x7FFFFFFFFFFFFFFF)
        return g

    def _get_env_origins(self):
        """Env origins (humanoid_env.py:586-611): terrain platforms, or a grid on the plane, as
        functions of the global env id."""
        off, total = self._global_ids()
        gid = torch.arange(off, off + self.num_envs)
        if self.custom_origins:
            max_init_level = self.cfg.terrain.max_init_terrain_level
            if not self.cfg.terrain.curriculum:
                max_init_level = self.cfg.terrain.num_rows - 1
            # levels/types live in the arena (int32): K_post's reset applies the curriculum
            self.terrain_levels = self._view(N.T["TERRAIN_LEVEL"])
            self.terrain_types = self._view(N.T["TERRAIN_TYPE"])
            levels = torch.randint(0, max_init_level + 1, (total,), generator=self._creation_generator(1))
            self.terrain_levels[:] = levels[off:off + self.num_envs].to(self.device, torch.int32)
            self.terrain_types[:] = torch.div(gid, (total / self.cfg.terrain.num_cols),
                                              rounding_mode="floor").to(self.device, torch.int32)
            self.max_terrain_level = self.cfg.terrain.num_rows
            self.env_origins[:] = self.terrain_origins[self.terrain_levels.long(), self.terrain_types.long()]
        else:
            num_cols = np.floor(np.sqrt(total))
            num_rows = np.ceil(total / num_cols)
            xx, yy = torch.meshgrid(torch.arange(num_rows), torch.arange(num_cols), indexing="ij")
            sp = self.cfg.env.env_spacing
            self.env_origins[:, 0] = (sp * xx.flatten()[gid]).to(self.device)
            self.env_origins[:, 1] = (sp * yy.flatten()[gid]).to(self.device)
            self.env_origins[:, 2] = 0.0

    def _randomize_props(self):
        """Creation-time DR (humanoid_env.py:528-553, 578-584): friction from 256 buckets, base mass;
        drawn for every global env and sliced to this shard."""
        dr = self.cfg.domain_rand
        off, total = self._global_ids()
        if dr.randomize_friction:
            lo, hi = dr.friction_range
            g = self._creation_generator(2)
            bucket_ids = torch.randint(0, 256, (total, 1), generator=g)[off:off + self.num_envs]
            buckets = (hi - lo) * torch.rand(256, 1, generator=g) + lo
            self.friction_coeffs = buckets[bucket_ids]
            self.env_frictions[:] = self.friction_coeffs.view(-1, 1).to(self.device)
        mass = np.full(self.num_envs, self._model.mass[0], dtype=np.float64)
        if dr.randomize_base_mass:
            lo, hi = dr.added_mass_range
            rs = np.random.RandomState((int(getattr(self.cfg, "seed", 5)) * 1000003 + 3) & 0xFFFFFFFF)
            mass += rs.uniform(lo, hi, size=total)[off:off + self.num_envs]
        self.body_mass[:] = torch.tensor(mass, dtype=torch.float32, device=self.device).view(-1, 1)

    def _init_buffers(self):
        self.common_step_counter = 0
        self.extras = {}
        self.gravity_vec = torch.tensor([0.0, 0.0, -1.0], device=self.device).repeat(self.num_envs, 1)
        self.forward_vec = torch.tensor([1.0, 0.0, 0.0], device=self.device).repeat(self.num_envs, 1)
        self.commands_scale = torch.tensor([self.obs_scales.lin_vel, self.obs_scales.lin_vel, self.obs_scales.ang_vel],
                                           device=self.device)
        self.p_gains = torch.tensor(self._aux["kp"], device=self.device).repeat(self.num_envs, 1)
        self.d_gains = torch.tensor(self._aux["kd"], device=self.device).repeat(self.num_envs, 1)
        self.torque_limits = torch.tensor(self._aux["torque_limits"], device=self.device)
        self.default_dof_pos = torch.tensor(self._aux["default_dof_pos"], device=self.device).unsqueeze(0)
        self.default_joint_pd_target = self.default_dof_pos.clone()
        lim = torch.tensor(self._aux["limits"], device=self.device)
        self.dof_pos_limits = lim * self.cfg.safety.pos_limit
        self.dof_vel_limits = torch.tensor(self._aux["velocity"], device=self.device) * self.cfg.safety.vel_limit
        self.base_init_state = torch.tensor(self.cfg.init_state.pos + self.cfg.init_state.rot + self.cfg.init_state.lin_vel
                                            + self.cfg.init_state.ang_vel, device=self.device)
        self.measured_heights = 0
        if self.cfg.terrain.measure_heights:
            self.height_points = self._init_height_points()
            self._height_xy = self.height_points[0, :, :2].contiguous()
            self.measured_heights = torch.zeros(self.num_envs, self.num_height_points, device=self.device)
        # extras["episode"] entries are views into a ring of this many post/reset snapshots
        self.episode_snapshot_rows = N.EP_RING
        self.course_gain = 1.0   # read by OnPolicyRunner.learn (on_policy_runner.py:160-162)
        self.course_ratio = 1.0

    def _init_height_points(self):
        """Base-frame sample grid (humanoid_env.py:314-328): [N, P, 3], x-major meshgrid."""
        y = torch.tensor(self.cfg.terrain.measured_points_y, device=self.device)
        x = torch.tensor(self.cfg.terrain.measured_points_x, device=self.device)
        grid_x, grid_y = torch.meshgrid(x, y, indexing="ij")
        self.num_height_points = grid_x.numel()
        points = torch.zeros(self.num_envs, self.num_height_points, 3, device=self.device)
        points[:, :, 0] = grid_x.flatten()
        points[:, :, 1] = grid_y.flatten()
        return points

    def _get_heights(self, env_ids=None):
        """Terrain heights under the sample grid (humanoid_env.py:949-985) by the HIP kernel
        hg_measure_heights: [N, P] (or [len(env_ids), P])."""
        mesh = self.cfg.terrain.mesh_type
        if mesh == "none":
            raise NameError("Can't measure height with terrain mesh type 'none'")
        if not hasattr(self, "height_points"):
            self.height_points = self._init_height_points()
            self._height_xy = self.height_points[0, :, :2].contiguous()
        out = torch.empty(self.num_envs, self.num_height_points, device=self.device)
        N.check(self.hg.hg_measure_heights(self.sim, ctypes.c_void_p(self._height_xy.data_ptr()),
                                           self.num_height_points, ctypes.c_void_p(out.data_ptr()), self._stream()),
                self.sim)
        if env_ids is not None and len(env_ids) > 0:
            return out[torch.as_tensor(env_ids, device=self.device, dtype=torch.long)]
        return out

    # ------------------------------------------------------------------ buffers with reference semantics
    @property
    def base_quat(self):
        return self.root_states[:, 3:7]

    @property
    def episode_length_buf(self):
        return self._ep_len

    @episode_length_buf.setter
    def episode_length_buf(self, value):
        # the runner re-assigns this attribute (on_policy_runner.py:104-107): copy into the sim
        self._ep_len.copy_(value.to(self._ep_len.dtype))

    @property
    def obs_buf(self):
        return self._obs_views[self.hg.hg_obs_head(self.sim)]

    @property
    def privileged_obs_buf(self):
        return self._priv_views[self.hg.hg_obs_head(self.sim)]

    @property
    def dof_state(self):
        """[N*D, 2] (pos, vel) — a copy: the sim stores dof state SoA."""
        return torch.stack((self.dof_pos, self.dof_vel), dim=-1).reshape(-1, 2)

    @property
    def ref_action(self):
        return 2 * self.ref_dof_pos

    # ------------------------------------------------------------------ hot path
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _publish_extras(self):
        # the latest post/reset launch left its EP_STATS snapshot in ring row hg_ep_stats_slot: a
        # view, intact for the next EP_RING - 1 launches (no copy kernel per step)
        # the per-term views of each ring row are built once and reused (22 fresh tensor views per
        # step cost ≈85 us of host time, a quarter of a policy step's GPU time)
        slot = self.hg.hg_ep_stats_slot(self.sim)
        cache = self.__dict__.setdefault("_ep_views", {})
        views = cache.get(slot)
        if views is None:
            stats = self._ep_ring[slot]
            views = cache[slot] = {"rew_" + n: stats[REWARD_NAMES.index(n)] for n in self.reward_names}
        self.extras = {"episode": dict(views), "time_outs": self.time_out_buf}

    def update_push_curriculum(self, iteration):
        """Push-recovery curriculum (config 5, BUILD-DEFINED): max push velocities ramp linearly
        from the configured values to *_final over push_curriculum_iterations PPO iterations.
        Called by OnPolicyRunner.learn once per iteration; no-op unless enabled."""
        dr = self.cfg.domain_rand
        if not getattr(dr, "push_curriculum", False):
            return
        f = min(1.0, max(0.0, iteration / max(1, int(dr.push_curriculum_iterations))))
        vxy = dr.max_push_vel_xy + f * (dr.max_push_vel_xy_final - dr.max_push_vel_xy)
        vang = dr.max_push_ang_vel + f * (dr.max_push_ang_vel_final - dr.max_push_ang_vel)
        if (self._hgcfg.max_push_vel_xy, self._hgcfg.max_push_ang_vel) != (np.float32(vxy), np.float32(vang)):
            self._hgcfg.max_push_vel_xy = vxy
            self._hgcfg.max_push_ang_vel = vang
            N.check(self.hg.hg_update_cfg(self.sim, ctypes.byref(self._hgcfg), self._stream()), self.sim)
        self.push_scale = (float(self._hgcfg.max_push_vel_xy), float(self._hgcfg.max_push_ang_vel))

    def _launch_reset(self, mask_u8):
        mp = ctypes.c_void_p(mask_u8.data_ptr()) if mask_u8 is not None else None
        N.check(self.hg.hg_reset_masked(self.sim, mp, ctypes.c_uint64(self.common_step_counter), self._stream()),
                self.sim)
        self._publish_extras()

    def step(self, actions):
        """humanoid_env.py:616-660."""
        if self.cfg.env.use_ref_actions:
            actions = actions + self.ref_action
        a = actions.detach()
        if a.dtype != torch.float32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
        if a.shape != (self.num_envs, self.num_actions):
            raise ValueError(f"actions must be [{self.num_envs}, {self.num_actions}], got {tuple(a.shape)}")
        s = self._stream()
        kt = self.kernel_timer
        if kt is not None:
            kt.start("k_step")
        N.check(self.hg.hg_step(self.sim, ctypes.c_void_p(a.data_ptr()), ctypes.c_uint64(self.common_step_counter), s),
                self.sim)
        if kt is not None:
            kt.stop("k_step")
            kt.start("k_post")
        self.common_step_counter += 1
        if self.cfg.terrain.measure_heights:
            # _post_physics_step_callback (:1012-1013): after physics, before termination/reset
            N.check(self.hg.hg_measure_heights(self.sim, ctypes.c_void_p(self._height_xy.data_ptr()),
                                               self.num_height_points, ctypes.c_void_p(self.measured_heights.data_ptr()),
                                               s), self.sim)
        sink, self._rollout_sink = self._rollout_sink, None
        if sink is not None:
            # this step's post launch also writes the rollout storage slot (hg_set_rollout_sink)
            vp = ctypes.c_void_p
            N.check(self.hg.hg_set_rollout_sink(self.sim, *[vp(t.data_ptr()) if t is not None else None
                                                             for t in sink]), self.sim)
        N.check(self.hg.hg_post(self.sim, ctypes.c_uint64(self.common_step_counter), s), self.sim)
        if kt is not None:
            kt.stop("k_post")
        self._publish_extras()
        if sink is not None:
            self.extras["rollout_sink"] = sink  # the slot tensors this step's post launch filled
        return self.get_observations(), self.get_privileged_observations(), self.rew_buf, self.reset_buf, self.extras

    _rollout_sink = None

    def set_rollout_sink(self, rewards, dones, time_outs=None):
        """The next step() also writes its rewards (float32), reset flags and time-out flags (uint8)
        into these [num_envs] device tensors — a PPO rollout-storage slot — inside its post launch
        (hg_set_rollout_sink), so the algorithm's storage write needs no launch of its own.  The
        step reports the tensors in extras["rollout_sink"]."""
        checks = [(rewards, torch.float32), (dones, torch.uint8)] + ([(time_outs, torch.uint8)] if time_outs is not None else [])
        for t, dt in checks:
            if (t is None or t.dtype != dt or t.device != self.device or t.numel() != self.num_envs
                    or not t.is_contiguous()):
                raise ValueError("set_rollout_sink: contiguous [num_envs] device tensors (float32 rewards, "
                                 "uint8 dones / time-outs)")
        self._rollout_sink = (rewards, dones, time_outs)

    def get_observations(self):
        return self.obs_buf.clone() if self.stable_observations else _live(self.obs_buf)

    def get_privileged_observations(self):
        return self.privileged_obs_buf.clone() if self.stable_observations else _live(self.privileged_obs_buf)

    def reset_idx(self, env_ids):
        """reset_idx (humanoid_env.py:1109-1163) for the given env ids, as a device mask; also
        refreshes the observation buffers of the reset envs."""
        if isinstance(env_ids, torch.Tensor) and env_ids.numel() == 0:
            return
        if len(env_ids) == 0:
            return
        mask = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
        mask[torch.as_tensor(env_ids, device=self.device, dtype=torch.long)] = 1
        self._launch_reset(mask)

    def compute_observations(self):
        raise NotImplementedError("observations are produced by hg_post inside step()")
