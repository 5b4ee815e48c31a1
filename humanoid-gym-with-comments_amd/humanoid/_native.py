"""ctypes binding of the hg_sim C ABI (include/hgsim.h).

This module is the Python side of the drop-in boundary: it mirrors the C structs, loads the
in-tree HIP library ``csrc/libhgsim.so`` and wraps arena sub-buffers as zero-copy torch tensors
(the role ``gymtorch.wrap_tensor`` plays in the reference, humanoid/envs/custom/humanoid_env.py:246-254).

There is deliberately NO CPU fallback: if the library or a GPU is missing, ``lib()`` raises.
"""
import ctypes
import json
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("HG_LIB") or os.path.join(PKG_ROOT, "csrc", "libhgsim.so")  # HG_LIB: diagnostic builds
MODEL_PATH = os.path.join(PKG_ROOT, "model", "xbotl_model.json")

HG_MAX_BODIES = 16
HG_MAX_DOF = 12
HG_MAX_CONTACTS = 24
HG_MAX_CAPSULES = 12
HG_MAX_PAIRS = 16
HG_NUM_REWARDS = 22
HG_LAMW = HG_MAX_CONTACTS * 3 + HG_MAX_PAIRS * 3 + 2 * HG_MAX_DOF

f32 = ctypes.c_float
i32 = ctypes.c_int32


class HgModel(ctypes.Structure):
    _fields_ = [
        ("num_bodies", i32), ("num_dof", i32), ("num_contacts", i32), ("num_foot_contacts", i32),
        ("num_leg_contacts", i32), ("num_capsules", i32), ("num_pairs", i32), ("_pad", i32),
        ("parent", i32 * HG_MAX_BODIES), ("contact_body", i32 * HG_MAX_CONTACTS),
        ("capsule_body", i32 * HG_MAX_CAPSULES), ("capsule_kind", i32 * HG_MAX_CAPSULES),
        ("pair", (i32 * 2) * HG_MAX_PAIRS),
        ("joint_pos", (f32 * 3) * HG_MAX_BODIES), ("joint_rot", (f32 * 9) * HG_MAX_BODIES),
        ("axis", (f32 * 3) * HG_MAX_BODIES), ("mass", f32 * HG_MAX_BODIES),
        ("com", (f32 * 3) * HG_MAX_BODIES), ("inertia", (f32 * 6) * HG_MAX_BODIES),
        ("armature", f32 * HG_MAX_BODIES), ("lower", f32 * HG_MAX_BODIES), ("upper", f32 * HG_MAX_BODIES),
        ("joint_friction", f32 * HG_MAX_BODIES),
        ("contact_pos", (f32 * 3) * HG_MAX_CONTACTS), ("contact_radius", f32 * HG_MAX_CONTACTS),
        ("capsule_p0", (f32 * 3) * HG_MAX_CAPSULES), ("capsule_p1", (f32 * 3) * HG_MAX_CAPSULES),
        ("capsule_radius", f32 * HG_MAX_CAPSULES),
    ]


class HgCfg(ctypes.Structure):
    _fields_ = [
        ("num_envs", i32), ("decimation", i32), ("pgs_iterations", i32), ("fix_base_link", i32),
        ("sim_dt", f32), ("gravity_z", f32), ("contact_offset", f32), ("max_depenetration_vel", f32),
        ("baumgarte", f32), ("ground_friction", f32),
        ("action_scale", f32), ("clip_actions", f32), ("dynamic_randomization", f32),
        ("kp", f32 * HG_MAX_DOF), ("kd", f32 * HG_MAX_DOF), ("torque_limit", f32 * HG_MAX_DOF),
        ("default_dof_pos", f32 * HG_MAX_DOF),
        ("terrain_type", i32), ("hf_rows", i32), ("hf_cols", i32),
        ("hf_horizontal_scale", f32), ("hf_vertical_scale", f32), ("hf_border", f32),
        ("heightfield", ctypes.c_void_p),
        ("frame_stack", i32), ("c_frame_stack", i32), ("max_episode_length", i32),
        ("resample_interval", i32), ("push_interval", i32),
        ("push_robots", i32), ("add_noise", i32), ("heading_command", i32), ("only_positive_rewards", i32),
        ("dt", f32), ("cycle_time", f32), ("target_joint_pos_scale", f32), ("target_feet_height", f32),
        ("base_height_target", f32), ("min_dist", f32), ("max_dist", f32), ("tracking_sigma", f32),
        ("max_contact_force", f32), ("max_push_vel_xy", f32), ("max_push_ang_vel", f32),
        ("cmd_lin_x", f32 * 2), ("cmd_lin_y", f32 * 2), ("cmd_ang_yaw", f32 * 2), ("cmd_heading", f32 * 2),
        ("noise_level", f32), ("noise_dof_pos", f32), ("noise_dof_vel", f32), ("noise_ang_vel", f32),
        ("noise_quat", f32),
        ("obs_lin_vel", f32), ("obs_ang_vel", f32), ("obs_dof_pos", f32), ("obs_dof_vel", f32), ("obs_quat", f32),
        ("clip_observations", f32),
        ("init_pos", f32 * 3), ("init_rot", f32 * 4), ("init_lin_vel", f32 * 3), ("init_ang_vel", f32 * 3),
        ("reward_scale", f32 * HG_NUM_REWARDS),
        ("feet_body", i32 * 2), ("knee_body", i32 * 2), ("ref_idx", i32 * 6), ("yaw_roll_idx", i32 * 4),
        ("seed", ctypes.c_uint64),
        ("curriculum", i32), ("terrain_rows", i32), ("terrain_cols", i32), ("terrain_env_length", f32),
        ("max_episode_length_s", f32), ("env_offset", i32), ("terrain_origins", ctypes.c_void_p),
    ]


class HgDesc(ctypes.Structure):
    _fields_ = [("offset_bytes", ctypes.c_size_t), ("dtype", i32), ("ndim", i32),
                ("shape", ctypes.c_int64 * 4), ("strides", ctypes.c_int64 * 4)]


# tensor ids (enum hg_tensor_id)
TENSOR_IDS = [
    "ROOT_STATE", "DOF_POS", "DOF_VEL", "CONTACT_FORCES", "RIGID_STATE", "TORQUES", "ACTIONS",
    "LAST_ACTIONS", "LAST_LAST_ACTIONS", "LAST_DOF_VEL", "LAST_ROOT_VEL", "COMMANDS", "OBS_BUF",
    "PRIV_BUF", "REW_BUF", "RESET_BUF", "TIME_OUT_BUF", "EPISODE_LENGTH", "EPISODE_SUMS",
    "FEET_AIR_TIME", "LAST_CONTACTS", "FEET_HEIGHT", "LAST_FEET_Z", "ENV_FRICTION", "BODY_MASS",
    "PUSH_FORCE", "PUSH_TORQUE", "BASE_LIN_VEL", "BASE_ANG_VEL", "PROJ_GRAVITY", "BASE_EULER",
    "REF_DOF_POS", "ENV_ORIGINS", "EP_STATS", "CONTACT_LAMBDA", "NONFINITE", "TERRAIN_LEVEL", "TERRAIN_TYPE",
    "EP_STATS_RING", "ROWS_DROPPED",
]
EP_RING = 64  # HG_EP_RING
T = {name: i for i, name in enumerate(TENSOR_IDS)}

# every symbol include/hgsim.h declares (checked by tests/test_boundary.py)
EXPORTS = ["hg_arena_bytes", "hg_create", "hg_destroy", "hg_last_error", "hg_tensor", "hg_step",
           "hg_post", "hg_set_rollout_sink", "hg_ep_stats_slot", "hg_obs_head", "hg_obs_window_advance", "hg_update_cfg", "hg_reset_masked", "hg_set_dof_state_indexed", "hg_set_root_state_indexed",
           "hg_set_root_state", "hg_set_env_props",
           "hg_measure_heights", "hg_gae_scan", "hg_gae_stats_len", "hg_gae_normalize", "hg_adam_step", "hg_adam_chunk", "hg_kl_mean", "hg_kl_lr_rule",
           "hg_rollout_act", "hg_rollout_act_head", "hg_rollout_act_tail", "hg_rollout_env", "hg_gather_rows", "hg_gather_rows_ex", "hg_gather_stacked", "hg_ppo_loss", "hg_ppo_loss_lr", "hg_ppo_loss_scratch", "hg_ppo_loss_backward",
           "hg_mlp_act_backward", "hg_mlp_act_backward_scratch", "hg_colsum_jobs", "hg_linear_skinny_supported",
           "hg_linear_skinny_forward", "hg_linear_skinny_backward", "hg_linear_skinny_backward_scratch",
           "hg_mlp_act_backward_bf16", "hg_linear_skinny_forward_bf16", "hg_linear_skinny_backward_bf16",
           "hg_cast_bf16_jobs", "hg_linear_act_forward", "hg_linear_act_tile", "hg_gemm_f32", "hg_gemm_tile",
           "hg_gemm_colpart_rows", "hg_gemm_f32_wgrad", "hg_gemm_x6_image_bytes", "hg_gemm_x6_image_jobs", "hg_gemm_x6_image_jobs_pitched", "hg_gemm_wgrad_img",
           "hg_gemm_f32_img", "hg_gemm_f32_img_split", "hg_gemm_splitk_kslice", "hg_gemm_f32_splitk", "hg_gemm_f32_splitk_img", "hg_linear_skinny_backward_act", "hg_linear_skinny_colpart_rows", "hg_version",
           "hg_source_hash"]

_LIB = None

DTYPE_CODES = {"float32": 0, "float16": 1, "bfloat16": 2}  # HG_DTYPE_* of include/hgsim.h


class GatherTable(ctypes.Structure):
    """hg_gather_table (include/hgsim.h)."""
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("width", ctypes.c_int64),
                ("src_dtype", ctypes.c_int32), ("dst_dtype", ctypes.c_int32)]


def source_hash(pkg_root=PKG_ROOT):
    """sha256 (first 16 hex digits) of the library's sources in the Makefile's stamp order (SRCS,
    csrc/hg_common.h, include/hgsim.h), as the Makefile computes it; None when the sources are
    not in the tree."""
    import hashlib
    try:
        with open(os.path.join(pkg_root, "Makefile")) as f:
            srcs = next(ln.split("=", 1)[1].split() for ln in f if ln.startswith("SRCS ="))
        h = hashlib.sha256()
        for rel in srcs + ["csrc/hg_common.h", "../include/hgsim.h"]:
            with open(os.path.join(pkg_root, rel), "rb") as f:
                h.update(f.read())
        return h.hexdigest()[:16]
    except (OSError, StopIteration):
        return None


def load_library(path=LIB_PATH):
    """Load libhgsim.so and declare signatures.  Raises if the HIP library is missing, or if it
    was built from other sources than the tree's (a stale binary: hg_source_hash)."""
    if not os.path.exists(path):
        raise RuntimeError(
            f"hg_sim HIP library not found at {path}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback on the product path)")
    # torch first, so libamdhip64.so.7 resolves to the runtime torch already loaded (one HIP runtime)
    import torch  # noqa: F401
    L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    L.hg_source_hash.restype = ctypes.c_char_p
    L.hg_source_hash.argtypes = []
    want = source_hash()
    if want is not None and path == os.path.join(PKG_ROOT, "csrc", "libhgsim.so"):
        got = L.hg_source_hash().decode()
        if got != want:
            raise RuntimeError(f"{path} was built from other sources (stamp {got}, tree {want}): rebuild it "
                               "(`make -C humanoid-gym-with-comments_amd`)")
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.hg_arena_bytes.restype = sz
    L.hg_arena_bytes.argtypes = [ctypes.POINTER(HgCfg)]
    L.hg_create.restype = ctypes.c_int
    L.hg_create.argtypes = [ctypes.POINTER(HgCfg), ctypes.POINTER(HgModel), vp, sz, ctypes.POINTER(vp)]
    L.hg_destroy.restype = None
    L.hg_destroy.argtypes = [vp]
    L.hg_last_error.restype = ctypes.c_char_p
    L.hg_last_error.argtypes = [vp]
    L.hg_tensor.restype = ctypes.c_int
    L.hg_tensor.argtypes = [vp, ctypes.c_int, ctypes.POINTER(HgDesc)]
    L.hg_step.restype = ctypes.c_int
    L.hg_step.argtypes = [vp, vp, ctypes.c_uint64, vp]
    L.hg_post.restype = ctypes.c_int
    L.hg_post.argtypes = [vp, ctypes.c_uint64, vp]
    L.hg_set_rollout_sink.restype = ctypes.c_int
    L.hg_set_rollout_sink.argtypes = [vp, vp, vp, vp]
    L.hg_update_cfg.restype = ctypes.c_int
    L.hg_update_cfg.argtypes = [vp, ctypes.POINTER(HgCfg), vp]
    L.hg_reset_masked.restype = ctypes.c_int
    L.hg_reset_masked.argtypes = [vp, vp, ctypes.c_uint64, vp]
    L.hg_set_dof_state_indexed.restype = ctypes.c_int
    L.hg_set_dof_state_indexed.argtypes = [vp, vp, ctypes.c_int, vp, vp, vp]
    L.hg_set_root_state_indexed.restype = ctypes.c_int
    L.hg_set_root_state_indexed.argtypes = [vp, vp, ctypes.c_int, vp, vp]
    L.hg_measure_heights.restype = ctypes.c_int
    L.hg_measure_heights.argtypes = [vp, vp, ctypes.c_int, vp, vp]
    L.hg_set_root_state.restype = ctypes.c_int
    L.hg_set_root_state.argtypes = [vp, vp, vp]
    L.hg_set_env_props.restype = ctypes.c_int
    L.hg_set_env_props.argtypes = [vp, vp, vp, vp]
    L.hg_gae_scan.restype = ctypes.c_int
    L.hg_gae_scan.argtypes = [vp, vp, vp, vp, vp, vp, vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                              ctypes.c_float, ctypes.c_int, vp]
    L.hg_gae_stats_len.restype = ctypes.c_int64
    L.hg_gae_stats_len.argtypes = [ctypes.c_int]
    L.hg_gae_normalize.restype = ctypes.c_int
    L.hg_gae_normalize.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int64, vp]
    L.hg_kl_mean.restype = ctypes.c_int
    L.hg_kl_mean.argtypes = [vp, vp, vp, vp, ctypes.c_int64, ctypes.c_int, vp, vp, vp]
    L.hg_kl_lr_rule.restype = ctypes.c_int
    L.hg_kl_lr_rule.argtypes = [vp, vp, vp, ctypes.c_double, ctypes.c_double, ctypes.c_double, vp]
    L.hg_rollout_act.restype = ctypes.c_int
    L.hg_rollout_act.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, vp, vp, vp, vp, vp, vp, ctypes.c_int64,
                                 vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, vp]
    L.hg_rollout_act_head.restype = ctypes.c_int
    L.hg_rollout_act_head.argtypes = [vp, ctypes.c_int64, vp, vp, ctypes.c_int] + L.hg_rollout_act.argtypes[1:]
    L.hg_rollout_act_tail.restype = ctypes.c_int
    L.hg_rollout_act_tail.argtypes = [vp, ctypes.c_int64, vp, vp, ctypes.c_int, vp, vp] + L.hg_rollout_act.argtypes[1:]
    L.hg_gather_stacked.restype = ctypes.c_int
    L.hg_gather_stacked.argtypes = [vp, ctypes.c_int64, vp, vp, vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.POINTER(GatherTable),
                                    ctypes.c_int, vp]
    L.hg_ep_stats_slot.restype = ctypes.c_int
    L.hg_ep_stats_slot.argtypes = [vp]
    L.hg_obs_head.restype = ctypes.c_int
    L.hg_obs_head.argtypes = [vp]
    L.hg_obs_window_advance.restype = ctypes.c_int
    L.hg_obs_window_advance.argtypes = [vp]
    L.hg_gather_rows_ex.restype = ctypes.c_int
    L.hg_gather_rows_ex.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(GatherTable), ctypes.c_int, vp]
    L.hg_gather_rows.restype = ctypes.c_int
    L.hg_gather_rows.argtypes = [vp, ctypes.c_int64, ctypes.c_int64] + [vp, vp, ctypes.c_int64, ctypes.c_int] * 3 + [vp]
    L.hg_rollout_env.restype = ctypes.c_int
    L.hg_rollout_env.argtypes = [vp, vp, vp, vp, ctypes.c_int, ctypes.c_float, vp, vp, vp, vp]
    L.hg_adam_chunk.restype = ctypes.c_int
    L.hg_adam_chunk.argtypes = []
    L.hg_ppo_loss.restype = ctypes.c_int
    L.hg_ppo_loss.argtypes = [vp, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                              ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_float, vp, vp, ctypes.c_int] + \
        [vp] * 6
    L.hg_ppo_loss_lr.restype = ctypes.c_int
    L.hg_ppo_loss_lr.argtypes = L.hg_ppo_loss.argtypes[:13] + [vp] * 5 + [vp, vp, ctypes.c_double, ctypes.c_double,
                                                                          ctypes.c_double, vp]
    L.hg_ppo_loss_scratch.restype = ctypes.c_int64
    L.hg_ppo_loss_scratch.argtypes = [ctypes.c_int64, ctypes.c_int]
    L.hg_ppo_loss_backward.restype = ctypes.c_int
    L.hg_ppo_loss_backward.argtypes = [vp, ctypes.c_int64, ctypes.c_int] + [vp] * 5
    L.hg_mlp_act_backward.restype = ctypes.c_int
    L.hg_mlp_act_backward.argtypes = [vp, vp, vp, ctypes.c_int64, ctypes.c_int, vp, vp, vp]
    L.hg_colsum_jobs.restype = ctypes.c_int
    L.hg_colsum_jobs.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64),
                                 ctypes.POINTER(ctypes.c_int), ctypes.c_int, vp]
    L.hg_mlp_act_backward_scratch.restype = ctypes.c_int64
    L.hg_mlp_act_backward_scratch.argtypes = [ctypes.c_int64, ctypes.c_int]
    L.hg_linear_act_forward.restype = ctypes.c_int
    L.hg_linear_act_forward.argtypes = [vp, ctypes.c_int64, vp, vp, vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]
    L.hg_linear_act_tile.restype = ctypes.c_int
    L.hg_linear_act_tile.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    L.hg_linear_skinny_supported.restype = ctypes.c_int
    L.hg_linear_skinny_supported.argtypes = [ctypes.c_int, ctypes.c_int]
    L.hg_linear_skinny_forward.restype = ctypes.c_int
    L.hg_linear_skinny_forward.argtypes = [vp, ctypes.c_int64, vp, vp, vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, vp]
    L.hg_linear_skinny_backward.restype = ctypes.c_int
    L.hg_linear_skinny_backward.argtypes = [vp, vp, ctypes.c_int64, vp, vp, vp, ctypes.c_int64, ctypes.c_int,
                                            ctypes.c_int, vp, vp]
    L.hg_linear_skinny_backward_scratch.restype = ctypes.c_int64
    L.hg_linear_skinny_backward_scratch.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    L.hg_mlp_act_backward_bf16.restype = ctypes.c_int
    L.hg_mlp_act_backward_bf16.argtypes = [vp, vp, vp, ctypes.c_int64, ctypes.c_int, vp, vp, vp]
    L.hg_linear_skinny_forward_bf16.restype = ctypes.c_int
    L.hg_linear_skinny_forward_bf16.argtypes = [vp, ctypes.c_int64, vp, vp, vp, ctypes.c_int64, ctypes.c_int,
                                                ctypes.c_int, vp]
    L.hg_linear_skinny_backward_bf16.restype = ctypes.c_int
    L.hg_linear_skinny_backward_bf16.argtypes = [vp, vp, ctypes.c_int64, vp, vp, vp, ctypes.c_int64, ctypes.c_int,
                                                 ctypes.c_int, vp, vp]
    L.hg_cast_bf16_jobs.restype = ctypes.c_int
    L.hg_cast_bf16_jobs.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64),
                                    ctypes.c_int, vp]
    L.hg_gemm_f32.restype = ctypes.c_int
    L.hg_gemm_f32.argtypes = [ctypes.c_int, vp, ctypes.c_int64, vp, ctypes.c_int64, vp, vp, ctypes.c_int64, vp,
                              ctypes.c_int64, vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]
    L.hg_gemm_f32_wgrad.restype = ctypes.c_int
    L.hg_gemm_f32_wgrad.argtypes = [vp, ctypes.c_int64, vp, ctypes.c_int64, vp, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    vp]
    L.hg_gemm_x6_image_bytes.restype = ctypes.c_int64
    L.hg_gemm_x6_image_bytes.argtypes = [ctypes.c_int64, ctypes.c_int64]
    L.hg_gemm_x6_image_jobs.restype = ctypes.c_int
    L.hg_gemm_x6_image_jobs.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(vp), ctypes.c_int, vp]
    L.hg_gemm_x6_image_jobs_pitched.restype = ctypes.c_int
    L.hg_gemm_x6_image_jobs_pitched.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64),
                                                ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int64),
                                                ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(vp),
                                                ctypes.POINTER(ctypes.c_int64), ctypes.c_int, vp]
    L.hg_gemm_f32_img_split.restype = ctypes.c_int
    L.hg_gemm_f32_img_split.argtypes = [vp, ctypes.c_int64, vp, vp, vp, vp, ctypes.c_int64, vp, ctypes.c_int64, ctypes.c_int,
                                        ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int64, vp]
    L.hg_gemm_splitk_kslice.restype = ctypes.c_int64
    L.hg_gemm_splitk_kslice.argtypes = [ctypes.c_int, ctypes.c_int]
    L.hg_gemm_f32_splitk.restype = ctypes.c_int
    L.hg_gemm_f32_splitk.argtypes = [vp, ctypes.c_int64, vp, ctypes.c_int64, vp, vp, ctypes.c_int64, vp, ctypes.c_int64,
                                     ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     vp]
    L.hg_gemm_f32_splitk_img.restype = ctypes.c_int
    L.hg_gemm_f32_splitk_img.argtypes = [vp, ctypes.c_int64, vp, ctypes.c_int64, vp, vp, ctypes.c_int64, vp,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, vp]
    L.hg_gemm_f32_img.restype = ctypes.c_int
    L.hg_gemm_f32_img.argtypes = [ctypes.c_int, vp, ctypes.c_int64, vp, vp, vp, vp, ctypes.c_int64, vp, ctypes.c_int64,
                                  vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int64, ctypes.c_int64, vp]
    L.hg_gemm_wgrad_img.restype = ctypes.c_int
    L.hg_gemm_wgrad_img.argtypes = [vp, vp, vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                    ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, vp]
    L.hg_gemm_tile.restype = ctypes.c_int
    L.hg_gemm_tile.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    L.hg_gemm_colpart_rows.restype = ctypes.c_int64
    L.hg_gemm_colpart_rows.argtypes = [ctypes.c_int64, ctypes.c_int]
    L.hg_linear_skinny_backward_act.restype = ctypes.c_int
    L.hg_linear_skinny_backward_act.argtypes = [vp, vp, ctypes.c_int64, vp, vp, vp, ctypes.c_int64, ctypes.c_int,
                                                ctypes.c_int, vp, vp]
    L.hg_linear_skinny_colpart_rows.restype = ctypes.c_int64
    L.hg_linear_skinny_colpart_rows.argtypes = [ctypes.c_int64]
    L.hg_version.restype = ctypes.c_char_p
    L.hg_version.argtypes = []
    return L


def lib():
    global _LIB
    if _LIB is None:
        _LIB = load_library()
    return _LIB


def check(status, handle=None):
    if status != 0:
        msg = lib().hg_last_error(handle)
        raise RuntimeError(f"hg_sim error {status}: {msg.decode() if msg else '?'}")


def stream_ptr(device):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr())


# ------------------------------------------------------------------------------------------------
# model table
# ------------------------------------------------------------------------------------------------
def load_model(path=MODEL_PATH, armature=0.0, joint_friction=True, self_collisions=True):
    """Build an HgModel from model/xbotl_model.json (output of tools/urdf_compile.py).

    armature: joint-space inertia added to every leg joint; the Isaac Gym asset option is 0
    (humanoid_config.py:118), which the simulator runs stably by treating the PD damping term
    implicitly.  0.01 kg m^2 is the robot's MJCF value (XBot-L.xml:37-39).
    joint_friction: apply the URDF's joint friction (0.1 N m on the ankles, XBot-L.urdf:1675-1677);
    or a dict {joint-name substring: friction N m} (last match wins, as the PD gain keys) that
    replaces it — the MJCF profile of scripts/sim2sim.py (frictionloss, XBot-L.xml:37-39,426).
    self_collisions: the self-collision pairs (asset.self_collisions = 0 enables them, :103):
    leg-vs-leg capsules, hands vs the thigh / shin of their side, the base-box bottom face vs the
    thighs.
    """
    with open(path) as f:
        js = json.load(f)
    m = HgModel()
    bodies = js["bodies"]
    m.num_bodies = len(bodies)
    m.num_dof = len(bodies) - 1
    for b, bd in enumerate(bodies):
        m.parent[b] = bd["parent"]
        m.mass[b] = bd["mass"]
        for i in range(3):
            m.com[b][i] = bd["com"][i]
        for i in range(6):
            m.inertia[b][i] = bd["inertia"][i]
        if b > 0:
            j = bd["joint"]
            for i in range(3):
                m.joint_pos[b][i] = j["origin_pos"][i]
                m.axis[b][i] = j["axis"][i]
            R = np.array(j["origin_rot"]).reshape(9)
            for i in range(9):
                m.joint_rot[b][i] = R[i]
            m.lower[b] = j["lower"]
            m.upper[b] = j["upper"]
            m.armature[b] = armature
            if isinstance(joint_friction, dict):
                f = 0.0
                for key, val in joint_friction.items():
                    if key in j["name"]:
                        f = float(val)
                m.joint_friction[b] = f
            else:
                m.joint_friction[b] = j.get("friction", 0.0) if joint_friction else 0.0
        else:
            for i in range(9):
                m.joint_rot[b][i] = 1.0 if i in (0, 4, 8) else 0.0
    cs = js["contacts"]
    if len(cs) > HG_MAX_CONTACTS:
        raise ValueError("too many contact candidates")
    m.num_contacts = len(cs)
    m.num_foot_contacts = sum(1 for c in cs if bodies[c["body"]]["name"].endswith("ankle_roll_link"))
    m.num_leg_contacts = js.get("num_leg_contacts", m.num_foot_contacts)
    for c, cd in enumerate(cs):
        m.contact_body[c] = cd["body"]
        m.contact_radius[c] = cd.get("radius", 0.0)
        for i in range(3):
            m.contact_pos[c][i] = cd["pos"][i]
    caps = js.get("capsules", [])
    m.num_capsules = len(caps)
    for k, cd in enumerate(caps):
        m.capsule_body[k] = cd["body"]
        m.capsule_kind[k] = cd.get("kind", 0)
        m.capsule_radius[k] = cd["radius"]
        for i in range(3):
            m.capsule_p0[k][i] = cd["p0"][i]
            m.capsule_p1[k][i] = cd["p1"][i]
    pairs = js.get("pairs", []) if self_collisions else []
    if len(pairs) > HG_MAX_PAIRS:
        raise ValueError("too many self-collision pairs")
    m.num_pairs = len(pairs)
    for p, (a, b) in enumerate(pairs):
        m.pair[p][0], m.pair[p][1] = a, b
    return m, js


def model_names(js):
    bodies = [b["name"] for b in js["bodies"]]
    dofs = [b["joint"]["name"] for b in js["bodies"][1:]]
    effort = [b["joint"]["effort"] for b in js["bodies"][1:]]
    limits = [(b["joint"]["lower"], b["joint"]["upper"]) for b in js["bodies"][1:]]
    velocity = [b["joint"]["velocity"] for b in js["bodies"][1:]]
    return bodies, dofs, effort, limits, velocity
