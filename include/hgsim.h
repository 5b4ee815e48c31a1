/*
 * hgsim.h — C ABI of the MI355X-native humanoid simulator ("hg_sim").
 *
 * This is the drop-in boundary that replaces, for the rollout + update hot path of
 * Rengar-Yang/humanoid-gym-with-comments, the Isaac Gym / PhysX tensor API and the eager-torch
 * env arithmetic.  Every entry point cites the reference interface it replaces (paths relative
 * to the reference repo root).  The Python facade (humanoid/envs/custom/humanoid_env.py in this
 * repo) binds it with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - All functions return int status (0 = HG_OK); no exceptions cross the ABI.  A per-handle
 *     message is available from hg_last_error().
 *   - Device memory is owned by the CALLER: hg_arena_bytes() says how many bytes the library
 *     needs, the caller allocates one device buffer (e.g. a torch uint8 tensor) and passes it to
 *     hg_create().  hg_tensor() returns offset/shape/strides of each named buffer inside that
 *     arena so the caller can wrap them zero-copy (what gymtorch.wrap_tensor did,
 *     humanoid_env.py:246-254).  Per-env state is SoA ([field][num_envs]).
 *   - All work is enqueued on the caller's stream (hipStream_t passed as void*), asynchronous
 *     to the host, with no host synchronisation inside any step/post/gae call.
 *   - The host API is not thread-safe per handle; one handle per GPU/process.
 */
#ifndef HGSIM_H
#define HGSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HG_OK 0
#define HG_ERR_ARG 1
#define HG_ERR_HIP 2
#define HG_ERR_STATE 3

#define HG_MAX_BODIES 16
#define HG_MAX_DOF 12
#define HG_MAX_CONTACTS 24  /* ground contact candidates (points / spheres) */
#define HG_MAX_CAPSULES 12
#define HG_MAX_PAIRS 16     /* self-collision capsule pairs */
#define HG_NUM_REWARDS 22
#define HG_MAX_TENSORS 32
/* solver warm-start impulses per env: 3 per ground candidate, 3 per pair, joint limits, joint friction */
#define HG_LAMW (HG_MAX_CONTACTS * 3 + HG_MAX_PAIRS * 3 + 2 * HG_MAX_DOF)

/* Articulated model table (output of tools/urdf_compile.py; replaces gym.load_asset +
 * get_asset_* queries, humanoid_env.py:455-470).  Body 0 is the floating base; body b>=1 is
 * attached to parent[b] by revolute joint (dof index b-1).  Frames follow URDF conventions.
 * Collision model (BUILD-DEFINED fits of the URDF collision meshes): ground contact candidates
 * are points (radius 0: sole corners, base-box corners) or spheres (capsule end caps); capsules
 * collide pairwise (self-collision, humanoid_config.py:103) with the normal from capsule
 * pair[p][0] to pair[p][1]; a capsule of kind 1 is the bottom face of the base-link box
 * (capsule_p0 / capsule_p1 = the face's corner extremes in the base frame, normal -z of the
 * base; it is only ever pair[p][0]), colliding with the closer end sphere of the other capsule.
 * Contact priority (the solver keeps at most 9 contact points per env): ground candidates
 * [0, num_leg_contacts), then the pairs, then the remaining candidates; num_contacts + num_pairs
 * <= 64 (detection runs one candidate per lane, two rounds over the env's 32 lanes). */
typedef struct hg_model {
  int32_t num_bodies;
  int32_t num_dof;
  int32_t num_contacts;      /* ground contact candidates */
  int32_t num_foot_contacts; /* the first num_foot_contacts candidates are foot-sole points */
  int32_t num_leg_contacts;  /* candidates ranked before the self-collision pairs */
  int32_t num_capsules;
  int32_t num_pairs;
  int32_t _pad;
  int32_t parent[HG_MAX_BODIES];
  int32_t contact_body[HG_MAX_CONTACTS];
  int32_t capsule_body[HG_MAX_CAPSULES];
  int32_t capsule_kind[HG_MAX_CAPSULES];  /* 0 capsule, 1 base-box bottom face */
  int32_t pair[HG_MAX_PAIRS][2];
  float joint_pos[HG_MAX_BODIES][3];   /* joint origin in parent-body frame */
  float joint_rot[HG_MAX_BODIES][9];   /* parent-body -> joint frame rotation, row-major */
  float axis[HG_MAX_BODIES][3];        /* joint axis in child frame */
  float mass[HG_MAX_BODIES];
  float com[HG_MAX_BODIES][3];         /* body frame */
  float inertia[HG_MAX_BODIES][6];     /* about COM, body frame: xx yy zz xy xz yz */
  float armature[HG_MAX_BODIES];       /* joint-space inertia added to M's diagonal (asset armature, 0) */
  float lower[HG_MAX_BODIES], upper[HG_MAX_BODIES];
  float joint_friction[HG_MAX_BODIES]; /* Coulomb friction torque bound, N m (URDF dynamics friction) */
  float contact_pos[HG_MAX_CONTACTS][3];
  float contact_radius[HG_MAX_CONTACTS];
  float capsule_p0[HG_MAX_CAPSULES][3], capsule_p1[HG_MAX_CAPSULES][3];  /* segment, body frame */
  float capsule_radius[HG_MAX_CAPSULES];
} hg_model;

/* Simulation + env-logic configuration.  Field meanings follow XBotLCfg
 * (humanoid/envs/custom/humanoid_config.py); comments give the source line. */
typedef struct hg_cfg {
  int32_t num_envs;
  int32_t decimation;          /* control.decimation :271 */
  int32_t pgs_iterations;      /* contact solver sweeps (PhysX TGS 4 pos + 1 vel :295-299) */
  int32_t fix_base_link;       /* asset.fix_base_link :116 */
  float sim_dt;                /* sim.dt :279 */
  float gravity_z;             /* sim.gravity :285 */
  float contact_offset;        /* physx.contact_offset :301 */
  float max_depenetration_vel; /* physx.max_depenetration_velocity :307 */
  float baumgarte;             /* build-defined position-error feedback fraction */
  float ground_friction;       /* terrain.static_friction :143 */
  /* actuation (humanoid_env.py:910-925) */
  float action_scale;          /* control.action_scale :264 */
  float clip_actions;          /* normalization.clip_actions :458 */
  float dynamic_randomization; /* domain_rand.dynamic_randomization :339 */
  float kp[HG_MAX_DOF], kd[HG_MAX_DOF], torque_limit[HG_MAX_DOF], default_dof_pos[HG_MAX_DOF];
  /* terrain: 0 plane, 1 heightfield (device int16 [hf_rows][hf_cols], row = x) */
  int32_t terrain_type;
  int32_t hf_rows, hf_cols;
  float hf_horizontal_scale, hf_vertical_scale, hf_border;
  const int16_t* heightfield;  /* device pointer, caller-owned; NULL for plane */
  /* env logic (humanoid_env.py:770-1163) */
  int32_t frame_stack, c_frame_stack;   /* env.frame_stack / c_frame_stack :43,45 */
  int32_t max_episode_length;           /* ceil(episode_length_s / dt) :187 */
  int32_t resample_interval;            /* resampling_time / dt :1012 */
  int32_t push_interval;                /* ceil(push_interval_s / dt) :191 */
  int32_t push_robots, add_noise, heading_command, only_positive_rewards;
  float dt;                             /* decimation * sim_dt */
  float cycle_time, target_joint_pos_scale, target_feet_height, base_height_target;
  float min_dist, max_dist, tracking_sigma, max_contact_force;
  float max_push_vel_xy, max_push_ang_vel;
  float cmd_lin_x[2], cmd_lin_y[2], cmd_ang_yaw[2], cmd_heading[2];
  float noise_level, noise_dof_pos, noise_dof_vel, noise_ang_vel, noise_quat;
  float obs_lin_vel, obs_ang_vel, obs_dof_pos, obs_dof_vel, obs_quat;
  float clip_observations;
  float init_pos[3], init_rot[4], init_lin_vel[3], init_ang_vel[3];
  float reward_scale[HG_NUM_REWARDS];   /* already multiplied by dt; alphabetical order */
  int32_t feet_body[2], knee_body[2];   /* [6,12], [4,10] */
  int32_t ref_idx[6];                   /* left pitch,knee,ankle ; right pitch,knee,ankle dofs */
  int32_t yaw_roll_idx[4];              /* default_joint_pos reward dof indices */
  uint64_t seed;
  /* terrain curriculum (_update_terrain_curriculum, humanoid_env.py:1075-1095); reset_idx
   * applies it before the root reset when curriculum != 0 and the step counter is non-zero
   * (the reference's init_done gate) */
  int32_t curriculum;
  int32_t terrain_rows, terrain_cols;   /* levels x types of terrain_origins */
  float terrain_env_length;             /* move up when the robot walked > length / 2 */
  float max_episode_length_s;           /* move down when it walked < |cmd_xy| * T_ep / 2 */
  int32_t env_offset;                   /* global id of this shard's env 0 (data parallel): every Philox
                                         * draw is keyed by the global env id */
  const float* terrain_origins;         /* device [rows, cols, 3], caller-owned */
} hg_cfg;

typedef struct hg_desc {
  size_t offset_bytes;  /* into the arena */
  int32_t dtype;        /* 0 f32, 1 i64, 2 u8(bool), 3 i32 */
  int32_t ndim;
  int64_t shape[4];
  int64_t strides[4];   /* in elements */
} hg_desc;

#define HG_EP_RING 64
/* tensor ids for hg_tensor() */
enum hg_tensor_id {
  HG_T_ROOT_STATE = 0,   /* [N,13] pos3 quat(xyzw)4 linvel3 angvel3, world   (actor_root_state) */
  HG_T_DOF_POS,          /* [N,D]                                            (dof_state[...,0]) */
  HG_T_DOF_VEL,          /* [N,D]                                            (dof_state[...,1]) */
  HG_T_CONTACT_FORCES,   /* [N,B,3] net contact force per body, world, SoA strides (1,3np,np) (net_contact_force) */
  HG_T_RIGID_STATE,      /* [N,B,13] per-body pos quat linvel angvel, SoA strides (1,13np,np) (rigid_body_state) */
  HG_T_TORQUES,          /* [N,D] last applied torques                       (self.torques) */
  HG_T_ACTIONS, HG_T_LAST_ACTIONS, HG_T_LAST_LAST_ACTIONS,
  HG_T_LAST_DOF_VEL, HG_T_LAST_ROOT_VEL,
  HG_T_COMMANDS,         /* [N,4] */
  HG_T_OBS_BUF,          /* [N, (frame_stack - 1 + HW) * 47] observation history window per env: the
                            stacked policy input is columns [h * 47, (h + frame_stack) * 47), h =
                            hg_obs_head() (a strided [N, frame_stack*47] view; HW = hg_obs_window_advance) */
  HG_T_PRIV_BUF,         /* [N, (c_frame_stack - 1 + HW) * 73], its stack columns [h * 73, (h + c_frame_stack) * 73) */
  HG_T_REW_BUF,          /* [N] */
  HG_T_RESET_BUF,        /* [N] bool */
  HG_T_TIME_OUT_BUF,     /* [N] bool */
  HG_T_EPISODE_LENGTH,   /* [N] int64 */
  HG_T_EPISODE_SUMS,     /* [22,N] */
  HG_T_FEET_AIR_TIME, HG_T_LAST_CONTACTS, HG_T_FEET_HEIGHT, HG_T_LAST_FEET_Z,
  HG_T_ENV_FRICTION, HG_T_BODY_MASS, HG_T_PUSH_FORCE, HG_T_PUSH_TORQUE,
  HG_T_BASE_LIN_VEL, HG_T_BASE_ANG_VEL, HG_T_PROJ_GRAVITY, HG_T_BASE_EULER,
  HG_T_REF_DOF_POS, HG_T_ENV_ORIGINS,
  HG_T_EP_STATS,         /* [22 + 2] episode reward means of the last resetting step, n_reset, any */
  HG_T_CONTACT_LAMBDA,   /* solver warm-start impulses [HG_LAMW, N] */
  HG_T_NONFINITE,        /* [N] int32 count of non-finite recoveries */
  HG_T_TERRAIN_LEVEL,    /* [N] int32 curriculum level (row of terrain_origins) */
  HG_T_TERRAIN_TYPE,     /* [N] int32 terrain type (column of terrain_origins) */
  HG_T_EP_STATS_RING,    /* [HG_EP_RING, 24] EP_STATS as left by each post/reset launch, launch k in row
                            k % HG_EP_RING (hg_ep_stats_slot): the per-step extras["episode"] snapshot
                            without a copy launch */
  HG_T_ROWS_DROPPED,     /* [N] int32: constraint rows / contact points the row budget dropped, summed over substeps;
                         * zero at hg_create, CUMULATIVE afterwards (resets do not clear it: zero it before a run) */
  HG_T_COUNT
};

/* ---- lifecycle ---- */
size_t hg_arena_bytes(const hg_cfg* cfg);
/* replaces gym.create_sim + _create_envs + prepare_sim (humanoid_env.py:333-524,
 * base_task.py:101-102).  *out_sim receives an opaque handle. */
int hg_create(const hg_cfg* cfg, const hg_model* model, void* arena, size_t arena_bytes,
              void** out_sim);
void hg_destroy(void* sim);
/* NULL sim -> last error of the most recent failed hg_create on this thread */
const char* hg_last_error(void* sim);
/* replaces acquire_*_tensor + gymtorch.wrap_tensor (humanoid_env.py:235-254) */
int hg_tensor(void* sim, int id, hg_desc* out);

/* ---- hot path ---- */
/* replaces the step() preamble + decimation x (_compute_torques, set_dof_actuation_force_tensor,
 * simulate, refresh_dof_state_tensor) + post-physics refreshes
 * (humanoid_env.py:620-649, 776-778).  actions: device [N,D] row-major, caller-owned. */
int hg_step(void* sim, const float* actions, uint64_t step_counter, void* stream);
/* replaces post_physics_step minus the refreshes (humanoid_env.py:780-806) and the obs clip
 * (:654-657): derived state, commands, push, termination, rewards, masked reset, observations.
 * common_step_counter is the reference's host-side counter (:781). */
/* ring row of HG_T_EP_STATS_RING written by the latest hg_post / hg_reset_masked launch (host-side
 * bookkeeping, no device access) */
int hg_ep_stats_slot(void* sim);
/* The rollout-storage slot the NEXT hg_post also fills: rewards_out[e] = the step's reward,
 * dones_out[e] = its reset flag, time_outs_out[e] (optional) = its time-out flag, e < num_envs —
 * what hg_rollout_env writes with the value bootstrap deferred (values == NULL), in extra blocks
 * of the post launch instead of a launch of its own (PPO.process_env_step, reference
 * ppo.py:127-138, then skips it).  One-shot: consumed by the next hg_post (hg_reset_masked leaves
 * it pending); all NULL clears it.  float32 / uint8 device arrays. */
int hg_set_rollout_sink(void* sim, float* rewards_out, uint8_t* dones_out, uint8_t* time_outs_out);
int hg_post(void* sim, uint64_t common_step_counter, void* stream);
/* first frame slot h of the current observation stacks in the HG_T_OBS_BUF / HG_T_PRIV_BUF
 * windows (host-side bookkeeping): every hg_post / hg_reset_masked advances it by one and writes
 * only the new frame; at h = HW - 1 the next launch moves the newest frame_stack - 1 frames to
 * slots 0.. and h restarts at 0.  Replaces the deque re-stacking of humanoid_env.py:880-887. */
int hg_obs_head(void* sim);
int hg_obs_window_advance(void* sim);
/* Runtime parameter update (curricula, e.g. the push-recovery ramp of config 5): copies *cfg into
 * the handle and, stream-ordered, into the device copy the kernels read.  Fields that size or
 * lay out the arena (num_envs, frame stacks, terrain tables, decimation) must be unchanged. */
int hg_update_cfg(void* sim, const hg_cfg* cfg, void* stream);
/* replaces reset_idx() (humanoid_env.py:1109-1163) for an explicit device mask [N] (u8). */
int hg_reset_masked(void* sim, const uint8_t* mask, uint64_t counter, void* stream);

/* ---- indexed state writes (replace set_*_tensor_indexed, humanoid_env.py:1046-1048,1070-1072,680-681) ---- */
/* env_ids: device int32 [n]; dof_pos/dof_vel: device [n,D]; root: device [n,13] */
int hg_set_dof_state_indexed(void* sim, const int32_t* env_ids, int n, const float* dof_pos,
                             const float* dof_vel, void* stream);
int hg_set_root_state_indexed(void* sim, const int32_t* env_ids, int n, const float* root, void* stream);
/* all envs (replaces set_actor_root_state_tensor, humanoid_env.py:680-681): root device [N,13] */
int hg_set_root_state(void* sim, const float* root, void* stream);
/* creation-time domain randomisation (replaces the friction / base-mass writes of
 * _process_rigid_shape_props / _process_rigid_body_props, humanoid_env.py:528-553,578-584):
 * friction, base_mass: device [N] f32 (either may be NULL) */
int hg_set_env_props(void* sim, const float* friction, const float* base_mass, void* stream);

/* ---- measured heights (replaces _get_heights, humanoid_env.py:949-985) ----
 * points_xy: device f32 [P,2] sample points in the base frame (the _init_height_points grid,
 * :314-328); out: device f32 [N,P].  Each point is yaw-rotated (quat_apply_yaw), offset by the
 * base position, quantised to the heightfield grid ((p + border) / horizontal_scale, truncated,
 * clipped to [0, rows-2] x [0, cols-2]) and reads min(h[i][j], h[i+1][j], h[i][j+1]) *
 * vertical_scale.  Zeros on a plane (terrain_type 0), as the reference. */
int hg_measure_heights(void* sim, const float* points_xy, int num_points, float* out, void* stream);

/* ---- rollout storage: fused GAE (replaces RolloutStorage.compute_returns,
 * humanoid/algo/ppo/rollout_storage.py:122-143) ---- */
/* Pass 1: reverse-time scan.  rewards/values/returns/advantages [T,N] f32, dones [T,N] u8,
 * last_values [N].  Writes returns and raw advantages, and adds (sum A, sum A^2) in float64 to
 * stats[0..1] (set instead of added when zero_stats != 0).  stats holds stats_len doubles, at
 * least hg_gae_stats_len(N): stats[2..] is scratch for the per-block partials, which are summed
 * in a fixed order (bitwise reproducible; no atomics).  Returns HG_ERR_ARG (1) without launching
 * when stats_len is too small.  Two launches. */
int hg_gae_scan(const float* rewards, const uint8_t* dones, const float* values,
                const float* last_values, float* returns, float* advantages, double* stats,
                int64_t stats_len, int T, int N, float gamma, float lam, int zero_stats, void* stream);
int64_t hg_gae_stats_len(int N);
/* Pass 2: advantages = (A - mean) / (std_unbiased + 1e-8) with mean/std from stats over
 * `count` elements (count = T*N*world_size after an all-reduce of stats). */
int hg_gae_normalize(float* advantages, const double* stats, int64_t count, int64_t n_local,
                     void* stream);

/* ---- rollout storage writes (replace the tail of PPO.act / process_env_step and
 * RolloutStorage.add_transitions, ppo.py:116-138, rollout_storage.py:83-100) ----
 * hg_rollout_act: actions = mean + std * N(0,1) (Philox keyed by seed, row_offset + row, counter:
 * the global env id under data parallelism), their
 * Normal log-prob summed over actions, mu, sigma, value, and the observation / critic
 * observation rows, all into storage slot t (obs_out/critic_obs_out fp32, or fp16 when
 * obs_fp16).  mean [N,A], std [A], value [N]: contiguous device f32; obs row r's columns
 * [obs_col0, obs_col0 + obs_width) at obs + r obs_ld (the newest frame only, for frame-only
 * storage: obs_col0 = (F - 1) W, obs_width = W) into obs_out rows obs_out_ld apart (0: packed,
 * obs_width), critic_obs [N, critic_width] rows at stride
 * critic_obs_ld (the envs' stacks are strided column slices of their history windows); value may
 * be NULL (values computed later in one batched critic pass).
 * hg_rollout_env: rewards_out = rewards + gamma * values * time_outs (time_outs may be NULL),
 * dones_out = reset; values == NULL defers the time-out bootstrap (rewards_out = rewards) and
 * time_outs_out (optional) keeps the time-out flags for it. */
int hg_rollout_act(const float* mean, const float* std, const float* value, const float* obs,
                   const float* critic_obs, int num_envs, int num_actions, int64_t obs_width,
                   int64_t critic_obs_width, int64_t obs_ld, int64_t obs_col0, int64_t critic_obs_ld,
                   float* actions_out, float* logp_out, float* mu_out, float* sigma_out, float* value_out,
                   void* obs_out, int64_t obs_out_ld, void* critic_obs_out, int obs_fp16, int row_offset,
                   uint64_t seed, uint64_t counter, void* stream);
/* hg_rollout_act with the policy's output layer fused in (the skinny 12 x 128 head of the actor,
 * replacing hg_linear_skinny_forward + the mean round trip): mean[r] = W h[r] + b computed by each
 * env's 16 sampling lanes with hg_linear_skinny_forward's arithmetic (bitwise its result), h [N,
 * head_k] rows h_ld apart (16-byte aligned, h_ld % 4 == 0), W [A, head_k], b [A]; the mean goes to
 * mu_out.  Supported: A == 12, head_k == 128 (else HG_ERR_ARG: run the two launches). */
int hg_rollout_act_head(const float* h, int64_t h_ld, const float* W, const float* b, int head_k, const float* std,
                        const float* value, const float* obs, const float* critic_obs, int num_envs, int num_actions,
                        int64_t obs_width, int64_t critic_obs_width, int64_t obs_ld, int64_t obs_col0,
                        int64_t critic_obs_ld, float* actions_out, float* logp_out, float* mu_out, float* sigma_out,
                        float* value_out, void* obs_out, int64_t obs_out_ld, void* critic_obs_out, int obs_fp16,
                        int row_offset, uint64_t seed, uint64_t counter, void* stream);
/* hg_rollout_act_head with the actor's last hidden layer folded in as well (one launch instead of
 * hg_linear_act_forward + hg_rollout_act_head): h = elu(x W3^T + b3) for x [N, tail_k] rows x_ld
 * apart, W3 [128, tail_k], b3 [128], computed as hg_linear_act_forward's 16 x 16 tile computes it
 * (the tile hg_linear_act_tile picks for the rollout's row counts: bitwise that launch pair's
 * result), kept on chip, then the head W [12, 128], b [12] and the sampling as in
 * hg_rollout_act_head.  16-byte aligned x / W3 / W, x_ld and tail_k multiples of 4, A == 12 (else
 * HG_ERR_ARG: run the two launches).  Replaces, with hg_rollout_act_head, ActorCritic.act's last
 * hidden layer + output layer (reference actor_critic.py:53-89, 111-121). */
int hg_rollout_act_tail(const float* x, int64_t x_ld, const float* W3, const float* b3, int tail_k, const float* W,
                        const float* b, const float* std, const float* value, const float* obs,
                        const float* critic_obs, int num_envs, int num_actions, int64_t obs_width,
                        int64_t critic_obs_width, int64_t obs_ld, int64_t obs_col0, int64_t critic_obs_ld,
                        float* actions_out, float* logp_out, float* mu_out, float* sigma_out, float* value_out,
                        void* obs_out, int64_t obs_out_ld, void* critic_obs_out, int obs_fp16, int row_offset,
                        uint64_t seed, uint64_t counter, void* stream);
int hg_rollout_env(const float* rewards, const uint8_t* reset, const uint8_t* time_outs, const float* values,
                   int num_envs, float gamma, float* rewards_out, uint8_t* dones_out, uint8_t* time_outs_out,
                   void* stream);

/* ---- minibatch gather (replaces the `observations.view(-1, ...)[batch_idx]` row gathers of
 * RolloutStorage.mini_batch_generator, rollout_storage.py:153-191) ----
 * dst_t[i, :] = src_t[idx[i], :] for up to three row-major tables (src1/src2 may be NULL) of
 * width_t elements of es_t bytes (4 or 2); idx values outside [0, src_rows) are clamped (the
 * caller's indices come from randperm).  One launch on `stream`, no host synchronisation. */
int hg_gather_rows(const int64_t* idx, int64_t rows, int64_t src_rows, const void* src0, void* dst0,
                   int64_t width0, int es0, const void* src1, void* dst1, int64_t width1, int es1,
                   const void* src2, void* dst2, int64_t width2, int es2, void* stream);

/* Typed form: per table the source and destination element types (HG_DTYPE_*); equal types copy,
 * fp16 -> bf16 and fp32 -> bf16 convert on the way (round-to-nearest-even) — the bf16 policy's
 * minibatch inputs gathered straight from fp16 / fp32 rollout storage.  1 <= ntab <= 3. */
enum { HG_DTYPE_F32 = 0, HG_DTYPE_F16 = 1, HG_DTYPE_BF16 = 2 };
typedef struct hg_gather_table {
  const void* src;
  void* dst;
  int64_t width;
  int32_t src_dtype;
  int32_t dst_dtype;
} hg_gather_table;
int hg_gather_rows_ex(const int64_t* idx, int64_t rows, int64_t src_rows, const hg_gather_table* tabs, int ntab,
                      void* stream);
/* Minibatch rows of a frame-only observation storage (replaces observations[batch_idx] when the
 * rollout keeps one frame per env-step, rollout_storage.py:153-191 with the stacking of
 * humanoid_env.py:880-887): dst[i] = the F*W stack of storage row s = idx[i] (t = s / N,
 * e = s % N) rebuilt from frames [N, T, W] (env-major: the newest frame of each slot's stack, a
 * row's frames one contiguous run), init [N, F*W] (slot 0's whole stack) and the u8 dones of
 * slot t, env e at dones[t dones_ts + e dones_es] (a reset at post step r zeroes the frames older
 * than slot r + 1's newest).  src_dtype F32 or F16 (frames and init), dst_dtype equal,
 * BF16, or F32 from F16.  1 <= F <= 64.  Up to two plain [T*N, width] tables (tabs, ntab <= 2, as
 * hg_gather_rows_ex) are gathered for the same rows by the same waves.  One launch, one wave per
 * row. */
int hg_gather_stacked(const int64_t* idx, int64_t rows, const void* frames, const void* init, const uint8_t* dones,
                      int64_t dones_ts, int64_t dones_es, int T, int N, int F, int W, int src_dtype, void* dst,
                      int dst_dtype, const hg_gather_table* tabs, int ntab, void* stream);

/* ---- PPO optimizer: fused global-norm clip + Adam (replaces
 * nn.utils.clip_grad_norm_(params, max_grad_norm); optimizer.step(), ppo.py:212-214) ----
 * A list of float32 device tensors (param, grad, Adam exp_avg / exp_avg_sq, per-tensor step
 * counter as a 1-float device scalar), split into fixed chunks of hg_adam_chunk() elements:
 * chunk_start[t] = first chunk of tensor t, chunk_start[count] = total chunks. */
typedef struct hg_tensor_list {
  int32_t count;
  int32_t _pad;
  float* param[HG_MAX_TENSORS];
  const float* grad[HG_MAX_TENSORS];
  float* exp_avg[HG_MAX_TENSORS];
  float* exp_avg_sq[HG_MAX_TENSORS];
  float* step[HG_MAX_TENSORS];
  int64_t numel[HG_MAX_TENSORS];
  int32_t chunk_start[HG_MAX_TENSORS + 1];
} hg_tensor_list;
/* lr: device float (read at run time, so a device-side LR schedule needs no host round trip);
 * max_norm <= 0 disables clipping; partial: device scratch of chunk_start[count] floats.
 * Deterministic (fixed-order reductions); two launches; graph-capturable. */
int hg_adam_step(const hg_tensor_list* tensors, const float* lr, float beta1, float beta2, float eps,
                 float max_norm, float* partial, void* stream);
int hg_adam_chunk(void);
/* Adaptive-KL learning rate (replaces the kl/lr block of ppo.py:162-176 on the device):
 * hg_kl_mean writes mean_rows sum_a KL(N(old_mu, old_sigma) || N(mu, sigma)) (the reference's
 * expression, with its 1e-5 inside the log) over [rows, num_actions] row-major inputs;
 * hg_kl_lr_rule applies lr /= 1.5 (floor lr_min) above 2*desired_kl, lr *= 1.5 (cap lr_max) in
 * (0, desired_kl/2), in float64 on lr64 and mirrors it into lr32.  Three launches in all. */
int hg_kl_mean(const float* mu, const float* sigma, const float* old_mu, const float* old_sigma, int64_t rows,
               int num_actions, float* kl_out, double* scratch /* >= ceil(rows/256) doubles */, void* stream);
int hg_kl_lr_rule(const float* kl, double* lr64, float* lr32, double desired_kl, double lr_min, double lr_max,
                  void* stream);

/* ---- fused PPO minibatch loss (replaces ppo.py:155-210 between the network outputs and
 * loss.backward(): log-prob, ratio, clipped surrogate, clipped value loss, entropy bonus,
 * lin-vel MSE, and the KL mean of the adaptive schedule) ----
 * Row-wise inputs are [rows, width] float32 with a row stride in elements (*_ld), so they may be
 * column slices of a packed table.  hg_ppo_loss writes
 *   loss_out[0] = surrogate + value_loss_coef*value_loss - entropy_coef*entropy
 *                 + lin_vel_coef*lin_vel_loss
 *   stats_out[0..3] = value_loss, surrogate_loss, lin_vel_loss, kl_mean
 * (accumulate_stats != 0: stats_out[0..2] += the three losses, stats_out[3] = kl_mean — the
 * running sums of an update need no extra launch)
 * and the gradients of loss_out[0] with respect to mu [rows, A], std [A], value [rows] and
 * lin_vel [rows, 3] (contiguous) — unscaled; hg_ppo_loss_backward multiplies them in place by
 * the device scalar grad_loss (the chain rule of loss.backward()).  Ties of torch.max and the
 * clamp boundaries follow torch's backward (max: half each on ties; clamp: pass-through on
 * [lo, hi]).  Deterministic: per-block partials, fixed-order float64 sums.  Two launches +
 * one for the backward; graph-capturable. */
typedef struct hg_ppo_batch {
  const float* mu;             int64_t mu_ld;             /* current policy mean  [rows, A] */
  const float* std;                                       /* current policy std   [A] */
  const float* value;          int64_t value_ld;          /* current critic value [rows] */
  const float* lin_vel;        int64_t lin_vel_ld;        /* lin-vel estimate     [rows, 3] */
  const float* lin_vel_target; int64_t lin_vel_target_ld; /* critic_obs[:, 53:56] */
  const float* actions;        int64_t actions_ld;        /* stored actions       [rows, A] */
  const float* old_logp;       int64_t old_logp_ld;
  const float* advantages;     int64_t advantages_ld;
  const float* target_values;  int64_t target_values_ld;
  const float* returns;        int64_t returns_ld;
  const float* old_mu;         int64_t old_mu_ld;
  const float* old_sigma;      int64_t old_sigma_ld;
} hg_ppo_batch;
int hg_ppo_loss(const hg_ppo_batch* batch, int64_t rows, int num_actions, float clip_lo, float clip_hi,
                float value_clip, int clipped_value_loss, float value_loss_coef, float entropy_coef,
                float lin_vel_coef, float* loss_out, float* stats_out, int accumulate_stats, float* grad_mu,
                float* grad_std,
                float* grad_value, float* grad_lin_vel, double* scratch /* >= hg_ppo_loss_scratch() doubles */,
                void* stream);
/* hg_ppo_loss with the adaptive-KL learning-rate rule (hg_kl_lr_rule, reference ppo.py:162-176)
 * applied in its final launch to this minibatch's KL mean (stats_out[3], read as hg_kl_lr_rule
 * reads it): lr64 / lr32 updated before the optimizer step of the same minibatch, one launch
 * fewer.  Single-process form: a data-parallel update applies hg_kl_lr_rule to the all-reduced
 * KL mean instead. */
int hg_ppo_loss_lr(const hg_ppo_batch* batch, int64_t rows, int num_actions, float clip_lo, float clip_hi,
                   float value_clip, int clipped_value_loss, float value_loss_coef, float entropy_coef,
                   float lin_vel_coef, float* loss_out, float* stats_out, int accumulate_stats, float* grad_mu,
                   float* grad_std, float* grad_value, float* grad_lin_vel, double* scratch, double* lr64,
                   float* lr32, double desired_kl, double lr_min, double lr_max, void* stream);
int64_t hg_ppo_loss_scratch(int64_t rows, int num_actions);
int hg_ppo_loss_backward(const float* grad_loss, int64_t rows, int num_actions, float* grad_mu, float* grad_std,
                         float* grad_value, float* grad_lin_vel, void* stream);

/* ---- policy MLP backward: activation backward + bias gradient in one pass (replaces, per
 * Linear(+ELU) layer of actor_critic.py:36-149, torch's ELU backward and grad_bias = gh.sum(0))
 * gh = gy * elu'(h) with elu'(h) = 1 for y > 0, y + 1 otherwise (y = the layer's ELU output);
 * y == NULL: identity activation, gh is gy (gh not written).  grad_bias[width] = column sums of
 * gh, deterministic (per-32-row tile partials in scratch, fixed-order column sums).
 * [rows, width] contiguous row-major float32; two launches.  grad_bias == NULL: one launch, the
 * [ceil(rows/32), width] partials are left in scratch for hg_colsum_jobs. */
int hg_mlp_act_backward(const float* gy, const float* y, float* gh, int64_t rows, int width, float* grad_bias,
                        float* scratch /* >= hg_mlp_act_backward_scratch() floats */, void* stream);
int64_t hg_mlp_act_backward_scratch(int64_t rows, int width);
/* Skinny output layers (n in {1,2,3,4,6,8,12,16}, k == 128): the last Linear of
 * each policy MLP (12 actions, 3 lin-vel, 1 value).  forward: y[rows, n] = x W^T + b, x rows of
 * stride ldx (16-byte aligned); backward: grad_wb = [dW (n x k row-major), db (n)] as
 * deterministic column sums over 64-row tiles, dx[rows, k] = gh W (dx may be NULL).  grad_wb ==
 * NULL: the [ceil(rows/64), n*k + n] partials are left in scratch for hg_colsum_jobs. */
int hg_linear_skinny_supported(int n, int k);
int hg_linear_skinny_forward(const float* x, int64_t ldx, const float* W, const float* b, float* y, int64_t rows,
                             int n, int k, void* stream);
int hg_linear_skinny_backward(const float* gh, const float* h, int64_t ldh, const float* W, float* dx,
                              float* grad_wb, int64_t rows, int n, int k,
                              float* scratch /* >= hg_linear_skinny_backward_scratch() floats */, void* stream);
int64_t hg_linear_skinny_backward_scratch(int64_t rows, int n, int k);
/* hg_linear_skinny_backward (dW / db partials left in scratch for hg_colsum_jobs) with the input
 * gradient fused with the ELU backward of the layer below (h is that layer's ELU output):
 * gh_prev[r][c] = (sum_j gh[r][j] W[j][c]) * (h[r][c] > 0 ? 1 : h[r][c] + 1), and colpart
 * [hg_linear_skinny_colpart_rows(rows), k] = its column sums per 64-row tile (the layer below's
 * bias-gradient partials, fixed order).  Replaces the skinny dX pass + hg_mlp_act_backward. */
int hg_linear_skinny_backward_act(const float* gh, const float* h, int64_t ldh, const float* W, float* gh_prev,
                                  float* colpart, int64_t rows, int n, int k,
                                  float* scratch /* >= hg_linear_skinny_backward_scratch() floats */, void* stream);
int64_t hg_linear_skinny_colpart_rows(int64_t rows);
/* bf16 policy (config 5, policy_dtype "bf16"): the same three passes with the activations,
 * activation gradients and hidden-layer inputs in bf16 (uint16_t bit patterns, round-to-nearest-
 * even), all accumulation, bias/weight-gradient partials, W of the skinny layer and its output y /
 * incoming gradient gh in float32.  Alignment: the bf16 arrays of the activation backward 8-byte,
 * skinny x rows 16-byte (ldx % 8 == 0), skinny h / dx 4-byte. */
int hg_mlp_act_backward_bf16(const uint16_t* gy, const uint16_t* y, uint16_t* gh, int64_t rows, int width,
                             float* grad_bias, float* scratch /* >= hg_mlp_act_backward_scratch() floats */,
                             void* stream);
int hg_linear_skinny_forward_bf16(const uint16_t* x, int64_t ldx, const float* W, const float* b, float* y,
                                  int64_t rows, int n, int k, void* stream);
int hg_linear_skinny_backward_bf16(const float* gh, const uint16_t* h, int64_t ldh, const float* W, uint16_t* dx,
                                   float* grad_wb, int64_t rows, int n, int k,
                                   float* scratch /* >= hg_linear_skinny_backward_scratch() floats */, void* stream);
/* dst[j][0..count[j]) = bf16(src[j][...]) for j < njobs <= 32, one launch (the bf16 copies of
 * the fp32 master weights a bf16 forward reads). */
int hg_cast_bf16_jobs(const float* const* src, uint16_t* const* dst, const int64_t* count, int njobs, void* stream);
/* Batched column sums (the deferred reductions of one MLP backward in one launch: bias-gradient
 * tile partials and split-K weight-gradient chunks, replacing per-layer grad.sum(0) launches):
 * dst[j][c] = sum over p < parts[j] of src[j][p * width[j] + c], fixed order, for j < njobs <= 16.
 * parts > 16 uses hg_mlp_act_backward's own final reduction (identical bits), except on wide jobs
 * (width >= 4096, a multiple of 4, 16-byte aligned: the split-K slices), which sum part p into
 * accumulator p % 8 and combine the eight as a fixed tree (parts <= 16: p = 0 .. parts-1 in order). */
int hg_colsum_jobs(const float* const* src, float* const* dst, const int64_t* width, const int* parts, int njobs,
                   void* stream);

/* Fused hidden-layer forward on the f32 matrix cores (replaces, per Linear + ELU pair of
 * actor_critic.py:36-149, torch's addmm + ELU): y[r][c] = act(sum_k x[r][k] W[c][k] + b[c]) for
 * r < rows, c < n; act 0 = identity, 1 = ELU(alpha 1).  x rows of stride ldx, W contiguous
 * [n, k] (both 4-byte aligned; 16-byte rows take the vector-load variant), b may be NULL, y rows
 * of stride ldy.  tile 0 = automatic wave tile, 1..5 = 64x64, 64x32, 32x64, 32x32 (32x32x2 MFMA),
 * 16x16 (16x16x4 MFMA).  One launch,
 * no host synchronisation, exact f32 products with f32 accumulation. */
int hg_linear_act_forward(const float* x, int64_t ldx, const float* W, const float* b, float* y, int64_t ldy,
                          int64_t rows, int n, int k, int act, int tile, void* stream);
int hg_linear_act_tile(int64_t rows, int n, int k);

/* LDS-staged f32 GEMM of the hidden layers with the layer's elementwise work in the epilogue
 * (replaces, per hidden layer of actor_critic.py:36-149, torch's addmm + ELU forward and, in the
 * backward, the input-gradient mm + the next lower layer's ELU backward + its bias-gradient sum):
 *   mode 0 (forward):    C[r][c] = act(sum_k A[r][k] B[c][k] + bias[c])      A [M, K] (lda), B [N, K] (ldb)
 *   mode 1 (input grad): C[r][c] = (sum_k A[r][k] B[k][c]) * elu'(Y[r][c])  A [M, K] (lda), B [K, N] (ldb)
 *   mode 3 (input grad, B given transposed: B [N, K] (ldb), bf16-split tiles only), as mode 1
 *     with elu'(from the ELU output y) = 1 for y > 0, y + 1 otherwise (act 1; act 0: no factor,
 *     Y unused); colpart (may be NULL) receives the column sums of C per row tile,
 *     [hg_gemm_colpart_rows(M, tile), N], reduced later in fixed order (hg_colsum_jobs).
 * tile 1..18 = f32-MFMA block tiles (exact f32 products, f32 accumulation, v_mfma_f32_32x32x2_f32);
 * tile 19..28 = the same product on the bf16 matrix cores with every f32 operand split exactly
 * into three bf16 terms and the six products of total order <= 2 accumulated in f32
 * (v_mfma_f32_32x32x16_bf16; error per element below torch's f32 GEMM's, csrc/hg_gemm.hip);
 * hg_gemm_tile picks one.  Rows of A, B, C 4-byte aligned (16-byte rows take the vector-load
 * staging).  One launch, no host synchronisation. */
int hg_gemm_f32(int mode, const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, const float* Y,
                int64_t ldY, float* C, int64_t ldc, float* colpart, int64_t M, int N, int K, int act, int tile,
                void* stream);
int hg_gemm_tile(int mode, int64_t M, int N, int K);
/* Weight gradient (replaces the dW = gh^T x matmuls of each Linear's backward): split-K slices
 * s < slices of the reduction over K rows, C + s * cstride [M, N] (ldc) =
 * sum_{k in slice s} A(m, k) B(n, k), with kmajor 0: A [K, M] (lda), B [K, N] (ldb) (the row-major
 * activations / gradients themselves), kmajor 1: A [M, K], B [N, K] (their transposes) — the
 * slices summed later in fixed order (hg_colsum_jobs).  tile 19..28 (the bf16-split kernels of
 * hg_gemm_f32). */
int hg_gemm_f32_wgrad(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                      int64_t cstride, int64_t M, int N, int64_t K, int slices, int kmajor, int tile, void* stream);
int64_t hg_gemm_colpart_rows(int64_t M, int tile);
/* Operand images of the bf16-split tiles (19..28): an f32 operand X with `rows` rows (the
 * product's M or N side) and reduction length K, split once into the three exact bf16 terms and
 * stored in the kernels' LDS fragment order (16-deep k chunks, count rounded up to even; three
 * planes; rows padded to a multiple of 256; zero past rows / K; csrc/hg_gemm.hip), so a GEMM block
 * copies its slice by LDS-DMA instead of loading, splitting and writing it per block tile.
 * Element (r, k) of X is P[r ld + k] (trans 0: k-contiguous rows — nn.Linear.weight as the
 * forward's B, activations / gradients as the A side) or P[k ld + r] (trans 1: reduction-major —
 * the weight [K, N] of the input grad, the row-major gh / x of the weight gradient).  One launch
 * for njobs <= 16 operands (arrays of njobs entries, host memory); img 16-byte aligned,
 * hg_gemm_x6_image_bytes(rows, K) bytes.  The image is tile-independent.  Routed: the weights
 * (B) only — split once per MLP call, 5-15 % off each GEMM; activation (A) and weight-gradient
 * images built by this separate pass cost more than they save (profiles/r3_gemm/x6_image_probe.jsonl). */
int64_t hg_gemm_x6_image_bytes(int64_t rows, int64_t K);
int hg_gemm_x6_image_jobs(const float* const* P, const int64_t* ld, const int* trans, const int64_t* rows,
                          const int64_t* K, void* const* img, int njobs, void* stream);
/* hg_gemm_x6_image_jobs writing row bands of shared images: pitch_rows[j] (> 0; <= 0 or a NULL
 * array: rows[j]) is the row count of the image job j writes into, img[j] = that image + the
 * band's first row x 32 bytes.  Jobs over the same K fill one image of the stacked rows, e.g. the
 * first layers of two MLPs reading the same input as one [n_a + n_b, K] forward operand (hg_mlp.py
 * mlp_pair_forward).  The bands of one image come as ONE chain of consecutive jobs (same
 * pitch_rows and K, each band starting where the previous one ends, in order) whose rows sum to
 * pitch_rows, every band but the last a multiple of 256 rows (each job zero-pads its band to a
 * multiple of 256 rows); anything else returns HG_ERR_ARG before any launch. */
int hg_gemm_x6_image_jobs_pitched(const float* const* P, const int64_t* ld, const int* trans, const int64_t* rows,
                                  const int64_t* K, void* const* img, const int64_t* pitch_rows, int njobs,
                                  void* stream);
/* hg_gemm_f32 modes 0 / 1 on a bf16-split tile with B from its image (Bimg: rows N, reduction K)
 * and A from its image (Aimg: rows M) or, Aimg NULL, staged from A (lda) as in hg_gemm_f32 — the
 * same epilogues and, bit for bit, the same result.  aimg_bytes / bimg_bytes: the images' sizes,
 * checked against hg_gemm_x6_image_bytes(M, K) / (N, K) (an image built for another shape is
 * refused; aimg_bytes is ignored when Aimg is NULL). */
int hg_gemm_f32_img(int mode, const float* A, int64_t lda, const void* Aimg, const void* Bimg, const float* bias,
                    const float* Y, int64_t ldY, float* C, int64_t ldc, float* colpart, int64_t M, int N, int K,
                    int act, int tile, int64_t aimg_bytes, int64_t bimg_bytes, void* stream);
/* hg_gemm_f32_img mode 0 (A staged from lda) writing its columns in two contiguous outputs: column
 * c < nsplit to C[r ldc + c] with bias[c], c >= nsplit to C2[r ldc2 + c - nsplit] with
 * bias2[c - nsplit] (nsplit a multiple of 256, 0 < nsplit < N; both biases or neither) — one GEMM
 * over two layers' stacked weights (hg_gemm_x6_image_jobs_pitched), each layer's bias and output
 * its own. */
int hg_gemm_f32_img_split(const float* A, int64_t lda, const void* Bimg, const float* bias, const float* bias2,
                          float* C, int64_t ldc, float* C2, int64_t ldc2, int nsplit, int64_t M, int N, int K, int act,
                          int tile, int64_t bimg_bytes, void* stream);
/* hg_gemm_f32_wgrad's split-K weight gradient from two images (Aimg: rows M, Bimg: rows N, both
 * with reduction K — build them with trans 1 from the row-major gh [K, M] and x [K, N]); the
 * slices start on 32-deep chunk pairs, ceil(K / slices) rounded up to a multiple of 32 rows each.
 * aimg_bytes / bimg_bytes as hg_gemm_f32_img. */
int hg_gemm_wgrad_img(const void* Aimg, const void* Bimg, float* C, int64_t ldc, int64_t cstride, int64_t M, int N,
                      int64_t K, int slices, int tile, int64_t aimg_bytes, int64_t bimg_bytes, void* stream);
/* Forward y = act(A W^T + bias) (the hidden-layer forward of actor_critic.py:53-89, as hg_gemm_f32
 * mode 0) in `slices` (2..16) split-K passes for few rows (the rollout's policy layers): the
 * bf16-split tile `tile` (20..28) writes slice s = sum over k in [s kslice, (s + 1) kslice)
 * (kslice = hg_gemm_splitk_kslice(K, slices); every slice non-empty) to ws + s M N (ws 16-byte
 * aligned, >= slices M N floats, dense [M, N] per slice), then a second launch writes
 * C[r ldc + c] = act(ws_0 + ... + ws_{S-1} + bias[c]), summed in slice order (deterministic).
 * A [M, K] (lda), W [N, K] (ldb) k-contiguous. */
int64_t hg_gemm_splitk_kslice(int K, int slices);
int hg_gemm_f32_splitk(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, float* C,
                       int64_t ldc, float* ws, int64_t ws_floats, int64_t M, int N, int K, int act, int tile,
                       int slices, void* stream);
/* hg_gemm_f32_splitk with W as its operand image (Bimg: hg_gemm_x6_image_jobs trans 0 of W [N, K],
 * bimg_bytes = hg_gemm_x6_image_bytes(N, K)): the slices read W's bf16 planes instead of splitting
 * W per block; bitwise the same C as hg_gemm_f32_splitk on the same tile.  Tiles 19..32 except 24,
 * 26, 29 (one 16-deep chunk per stage).  The rollout builds the image once per weight update. */
int hg_gemm_f32_splitk_img(const float* A, int64_t lda, const void* Bimg, int64_t bimg_bytes, const float* bias,
                           float* C, int64_t ldc, float* ws, int64_t ws_floats, int64_t M, int N, int K, int act,
                           int tile, int slices, void* stream);

/* library build info; hg_source_hash: first 16 hex digits of the sha256 of the sources the
 * library was built from (the Makefile's SRCS, csrc/hg_common.h, include/hgsim.h, concatenated) */
const char* hg_version(void);
const char* hg_source_hash(void);

#ifdef __cplusplus
}
#endif
#endif /* HGSIM_H */
