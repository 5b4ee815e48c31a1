// hg_api.hip — host side of the hg_sim C ABI (include/hgsim.h): arena layout, tensor
// descriptors, launches.  No host synchronisation on any step/post path.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "hg_common.h"

extern "C" int hg_launch_step(const HgState* S, const hg_cfg* hcfg, const float* actions, uint64_t step_counter,
                               hipStream_t stream);
extern "C" int hg_launch_post(const HgState* S, const hg_cfg* hcfg, uint64_t counter, int mode, const uint8_t* mask,
                              float* frame_obs, float* frame_priv, HgWindow obs, HgWindow priv, float inv_len_s,
                              int ep_slot, HgSink sink, hipStream_t stream);

namespace {

thread_local std::string g_create_error;

struct Field {
  int id;
  int dtype;      // 0 f32, 1 i64, 2 u8, 3 i32
  int rows;       // SoA rows per env (ignored for special)
  int ndim;       // view ndim
  int64_t shp[3]; // trailing dims of the [N, ...] view (row index = r0*shp... see make_desc)
};

size_t esize(int dtype) { return dtype == 1 ? 8 : (dtype == 2 ? 1 : 4); }
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Layout {
  size_t off[HG_T_COUNT + 8];
  size_t bytes;
  // extra regions
  size_t obs_buf, priv_buf, frame_obs, frame_priv, cfg, model, obs_noise, noise_counter, env_rows, env_order;
};

enum { X_OBS0 = HG_T_COUNT, X_OBS1, X_PRIV0, X_PRIV1, X_FOBS, X_FPRIV, X_CFG, X_MODEL };

int soa_rows(int id) {
  switch (id) {
    case HG_T_ROOT_STATE: return 13;
    case HG_T_DOF_POS: case HG_T_DOF_VEL: case HG_T_TORQUES: case HG_T_ACTIONS: case HG_T_LAST_ACTIONS:
    case HG_T_LAST_LAST_ACTIONS: case HG_T_LAST_DOF_VEL: case HG_T_REF_DOF_POS: return HG_ND;
    case HG_T_CONTACT_FORCES: return HG_NB * 3;
    case HG_T_RIGID_STATE: return HG_NB * 13;
    case HG_T_LAST_ROOT_VEL: return 6;
    case HG_T_COMMANDS: return 4;
    case HG_T_REW_BUF: case HG_T_RESET_BUF: case HG_T_TIME_OUT_BUF: case HG_T_EPISODE_LENGTH:
    case HG_T_ENV_FRICTION: case HG_T_BODY_MASS: case HG_T_NONFINITE: case HG_T_TERRAIN_LEVEL:
    case HG_T_TERRAIN_TYPE: case HG_T_ROWS_DROPPED: return 1;
    case HG_T_EPISODE_SUMS: return HG_NUM_REWARDS;
    case HG_T_FEET_AIR_TIME: case HG_T_LAST_CONTACTS: case HG_T_FEET_HEIGHT: case HG_T_LAST_FEET_Z: return 2;
    case HG_T_PUSH_FORCE: case HG_T_PUSH_TORQUE: case HG_T_BASE_LIN_VEL: case HG_T_BASE_ANG_VEL:
    case HG_T_PROJ_GRAVITY: case HG_T_BASE_EULER: case HG_T_ENV_ORIGINS: return 3;
    case HG_T_CONTACT_LAMBDA: return HG_LAMW;
    default: return 0;
  }
}
int dtype_of(int id) {
  switch (id) {
    case HG_T_RESET_BUF: case HG_T_TIME_OUT_BUF: case HG_T_LAST_CONTACTS: return 2;
    case HG_T_EPISODE_LENGTH: return 1;
    case HG_T_NONFINITE: case HG_T_TERRAIN_LEVEL: case HG_T_TERRAIN_TYPE: case HG_T_ROWS_DROPPED: return 3;
    default: return 0;
  }
}

// Observation histories as sliding windows: env row e holds F - 1 + HW frame slots; the current
// stack (the policy input) is slots [head, head + F), head advancing by one per post launch, so a
// step writes one frame per env instead of re-copying the whole stack.  When head reaches HW the
// newest F - 1 frames move to slots 0 .. F - 2 in the same launch (once every HW steps).  HW is
// shared by both tables, >= 26 and >= F - 1 of each.
int win_advance(const hg_cfg* c) { return std::max(26, std::max(c->frame_stack, c->c_frame_stack) - 1); }
int win_frames(int F, const hg_cfg* c) { return F - 1 + win_advance(c); }

Layout make_layout(const hg_cfg* c) {
  Layout L;
  const int n = c->num_envs;
  const int np = (n + 63) & ~63;
  size_t o = 0;
  for (int id = 0; id < HG_T_COUNT; id++) {
    L.off[id] = o;
    if (id == HG_T_OBS_BUF || id == HG_T_PRIV_BUF) continue;  // below
    // EP_STATS region: [24] stats, [24] accumulators, then the [HG_EP_RING, 24] snapshot ring
    if (id == HG_T_EP_STATS) { o += align256((48 + HG_EP_RING * 24) * sizeof(float)); continue; }
    if (id == HG_T_EP_STATS_RING) { L.off[id] = L.off[HG_T_EP_STATS] + 48 * sizeof(float); continue; }
    o += align256((size_t)soa_rows(id) * np * esize(dtype_of(id)));
  }
  // the observation histories: one sliding window per env row (hg_obs_window_frames)
  const size_t ob = (size_t)n * win_frames(c->frame_stack, c) * HG_OBS1 * 4;
  const size_t pb = (size_t)n * win_frames(c->c_frame_stack, c) * HG_PRIV1 * 4;
  L.obs_buf = o; o += align256(ob);
  L.priv_buf = o; o += align256(pb);
  L.frame_obs = o; o += align256((size_t)n * HG_OBS1 * 4);
  L.frame_priv = o; o += align256((size_t)n * HG_PRIV1 * 4);
  L.cfg = o; o += align256(sizeof(hg_cfg));
  L.model = o; o += align256(sizeof(hg_model));
  L.obs_noise = o; o += align256((size_t)48 * np * 4);
  L.noise_counter = o; o += align256(sizeof(uint64_t));
  L.env_rows = o; o += align256((size_t)np * 4);
  L.env_order = o; o += align256((size_t)np * 4);
  L.off[HG_T_OBS_BUF] = L.obs_buf;
  L.off[HG_T_PRIV_BUF] = L.priv_buf;
  L.bytes = o;
  return L;
}

struct Sim {
  hg_cfg cfg;
  hg_model model;
  char* arena;
  size_t bytes;
  Layout L;
  HgState S;
  int head;    // first window slot of the current observation stack
  uint64_t post_seq = 0;  // post/reset launches so far: EP_STATS ring row of the next one
  int ep_slot = 0;        // ring row written by the latest one
  HgSink sink{nullptr, nullptr, nullptr};  // one-shot: consumed by the next hg_post
  std::string err;
};

int fail(Sim* s, int code, const std::string& m) {
  if (s) s->err = m; else g_create_error = m;
  return code;
}

__global__ void k_init(HgState S) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S.n) return;
  const hg_cfg* c = S.cfg;
  const int np = S.np;
  for (int i = 0; i < 3; i++) S.root[i * np + e] = c->init_pos[i] + S.env_origins[i * np + e];
  for (int i = 0; i < 4; i++) S.root[(3 + i) * np + e] = c->init_rot[i];
  for (int i = 0; i < 3; i++) {
    S.root[(7 + i) * np + e] = c->init_lin_vel[i];
    S.root[(10 + i) * np + e] = c->init_ang_vel[i];
  }
  for (int j = 0; j < HG_ND; j++) S.dof_pos[j * np + e] = c->default_dof_pos[j];
  S.last_feet_z[0 * np + e] = 0.05f;  // self.last_feet_z = 0.05 (humanoid_env.py:175)
  S.last_feet_z[1 * np + e] = 0.05f;
  S.body_mass[e] = S.model->mass[0];
  S.friction[e] = 1.0f;
  S.proj_gravity[2 * np + e] = -1.0f;
  S.reset_buf[e] = 1;
  S.env_order[e] = e;  // identity until the first step has counted rows
}

}  // namespace

extern "C" {

size_t hg_arena_bytes(const hg_cfg* cfg) {
  if (!cfg || cfg->num_envs <= 0) return 0;
  return make_layout(cfg).bytes;
}

int hg_create(const hg_cfg* cfg, const hg_model* model, void* arena, size_t arena_bytes, void** out_sim) {
  if (!cfg || !model || !arena || !out_sim) return fail(nullptr, HG_ERR_ARG, "null argument");
  if (cfg->num_envs <= 0) return fail(nullptr, HG_ERR_ARG, "num_envs must be > 0");
  if (model->num_bodies != HG_NB || model->num_dof != HG_ND)
    return fail(nullptr, HG_ERR_ARG, "model must have 13 bodies / 12 dofs (XBot-L profile)");
  if (model->num_contacts <= 0 || model->num_contacts > HG_MAX_CONTACTS) return fail(nullptr, HG_ERR_ARG, "bad contact count");
  if (model->num_pairs < 0 || model->num_pairs > HG_MAX_PAIRS || model->num_capsules < 0 ||
      model->num_capsules > HG_MAX_CAPSULES || model->num_contacts + model->num_pairs > 64 ||
      model->num_leg_contacts < 0 || model->num_leg_contacts > model->num_contacts)
    return fail(nullptr, HG_ERR_ARG, "bad collision model (<= 64 contact candidates + pairs)");
  for (int p = 0; p < model->num_pairs; p++) {
    for (int s = 0; s < 2; s++)
      if (model->pair[p][s] < 0 || model->pair[p][s] >= model->num_capsules)
        return fail(nullptr, HG_ERR_ARG, "pair names a missing capsule");
    if (model->capsule_kind[model->pair[p][1]] != 0 || model->capsule_kind[model->pair[p][0]] < 0 ||
        model->capsule_kind[model->pair[p][0]] > 1 ||
        (model->capsule_kind[model->pair[p][0]] == 1 && model->capsule_body[model->pair[p][0]] != 0))
      return fail(nullptr, HG_ERR_ARG, "a box-face primitive (kind 1, on the base) may only be a pair's first shape");
  }
  for (int b = 1; b < HG_NB; b++)  // two 6-link leg chains off the base (XBot-L topology)
    if (model->parent[b] != ((b == 1 || b == 7) ? 0 : b - 1))
      return fail(nullptr, HG_ERR_ARG, "model topology must be base + two 6-link leg chains (bodies 1-6, 7-12)");
  if (cfg->decimation <= 0 || cfg->sim_dt <= 0.f || cfg->frame_stack <= 0 || cfg->c_frame_stack <= 0)
    return fail(nullptr, HG_ERR_ARG, "bad timing / stacking config");
  if (cfg->resample_interval <= 0 || cfg->push_interval <= 0) return fail(nullptr, HG_ERR_ARG, "bad intervals");
  if (cfg->terrain_type != 0 && (!cfg->heightfield || cfg->hf_rows < 2 || cfg->hf_cols < 2))
    return fail(nullptr, HG_ERR_ARG, "heightfield terrain needs a device heightfield");
  if (cfg->curriculum && (!cfg->terrain_origins || cfg->terrain_rows < 1 || cfg->terrain_cols < 1))
    return fail(nullptr, HG_ERR_ARG, "terrain curriculum needs the device terrain_origins table");
  Sim* s = new Sim();
  s->cfg = *cfg;
  s->model = *model;
  s->L = make_layout(cfg);
  if (arena_bytes < s->L.bytes) {
    delete s;
    return fail(nullptr, HG_ERR_ARG, "arena too small");
  }
  if (((uintptr_t)arena & 255) != 0) {
    delete s;
    return fail(nullptr, HG_ERR_ARG, "arena must be 256-byte aligned");
  }
  s->arena = (char*)arena;
  s->bytes = arena_bytes;
  s->head = 0;
  const int n = cfg->num_envs;
  HgState& S = s->S;
  S.n = n;
  S.np = (n + 63) & ~63;
  auto P = [&](int id) { return (void*)(s->arena + s->L.off[id]); };
  S.root = (float*)P(HG_T_ROOT_STATE);
  S.dof_pos = (float*)P(HG_T_DOF_POS);
  S.dof_vel = (float*)P(HG_T_DOF_VEL);
  S.contact = (float*)P(HG_T_CONTACT_FORCES);
  S.rigid = (float*)P(HG_T_RIGID_STATE);
  S.torques = (float*)P(HG_T_TORQUES);
  S.actions = (float*)P(HG_T_ACTIONS);
  S.last_actions = (float*)P(HG_T_LAST_ACTIONS);
  S.last_last_actions = (float*)P(HG_T_LAST_LAST_ACTIONS);
  S.last_dof_vel = (float*)P(HG_T_LAST_DOF_VEL);
  S.last_root_vel = (float*)P(HG_T_LAST_ROOT_VEL);
  S.commands = (float*)P(HG_T_COMMANDS);
  S.obs = (float*)(s->arena + s->L.obs_buf);
  S.priv = (float*)(s->arena + s->L.priv_buf);
  S.rew = (float*)P(HG_T_REW_BUF);
  S.reset_buf = (uint8_t*)P(HG_T_RESET_BUF);
  S.time_out = (uint8_t*)P(HG_T_TIME_OUT_BUF);
  S.ep_len = (int64_t*)P(HG_T_EPISODE_LENGTH);
  S.ep_sums = (float*)P(HG_T_EPISODE_SUMS);
  S.feet_air_time = (float*)P(HG_T_FEET_AIR_TIME);
  S.last_contacts = (uint8_t*)P(HG_T_LAST_CONTACTS);
  S.feet_height = (float*)P(HG_T_FEET_HEIGHT);
  S.last_feet_z = (float*)P(HG_T_LAST_FEET_Z);
  S.friction = (float*)P(HG_T_ENV_FRICTION);
  S.body_mass = (float*)P(HG_T_BODY_MASS);
  S.push_force = (float*)P(HG_T_PUSH_FORCE);
  S.push_torque = (float*)P(HG_T_PUSH_TORQUE);
  S.base_lin_vel = (float*)P(HG_T_BASE_LIN_VEL);
  S.base_ang_vel = (float*)P(HG_T_BASE_ANG_VEL);
  S.proj_gravity = (float*)P(HG_T_PROJ_GRAVITY);
  S.base_euler = (float*)P(HG_T_BASE_EULER);
  S.ref_dof_pos = (float*)P(HG_T_REF_DOF_POS);
  S.env_origins = (float*)P(HG_T_ENV_ORIGINS);
  S.ep_stats = (float*)P(HG_T_EP_STATS);
  S.lambda = (float*)P(HG_T_CONTACT_LAMBDA);
  S.nonfinite = (int32_t*)P(HG_T_NONFINITE);
  S.terrain_level = (int32_t*)P(HG_T_TERRAIN_LEVEL);
  S.terrain_type = (int32_t*)P(HG_T_TERRAIN_TYPE);
  S.rows_dropped = (int32_t*)P(HG_T_ROWS_DROPPED);
  S.cfg = (const hg_cfg*)(s->arena + s->L.cfg);
  S.model = (const hg_model*)(s->arena + s->L.model);
  S.obs_noise = (float*)(s->arena + s->L.obs_noise);
  S.noise_counter = (uint64_t*)(s->arena + s->L.noise_counter);
  S.env_rows = (int32_t*)(s->arena + s->L.env_rows);
  S.env_order = (int32_t*)(s->arena + s->L.env_order);
  {
    // K_step's wave balancing (hg_common.h hg_env_order_block, run by the post launch): on unless HG_WAVE_BALANCE=0
    const char* wb = getenv("HG_WAVE_BALANCE");
    S.balance = (wb && wb[0] == '0') ? 0 : 1;
  }
  // zero the arena, upload cfg/model, initial state (synchronous: creation is not on the hot path)
  if (hipMemset(arena, 0, s->L.bytes) != hipSuccess ||
      hipMemcpy((void*)S.cfg, &s->cfg, sizeof(hg_cfg), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy((void*)S.model, &s->model, sizeof(hg_model), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(S.noise_counter, 0xFF, sizeof(uint64_t)) != hipSuccess) {
    delete s;
    return fail(nullptr, HG_ERR_HIP, "hip memset/memcpy failed (is the arena device memory?)");
  }
  hipLaunchKernelGGL(k_init, dim3((n + 255) / 256), dim3(256), 0, 0, S);
  if (hipDeviceSynchronize() != hipSuccess) {
    delete s;
    return fail(nullptr, HG_ERR_HIP, "init kernel failed");
  }
  *out_sim = s;
  return HG_OK;
}

void hg_destroy(void* sim) { delete (Sim*)sim; }

const char* hg_last_error(void* sim) {
  if (!sim) return g_create_error.c_str();
  return ((Sim*)sim)->err.c_str();
}

int hg_tensor(void* sim, int id, hg_desc* d) {
  Sim* s = (Sim*)sim;
  if (!s || !d || id < 0 || id >= HG_T_COUNT) return fail(s, HG_ERR_ARG, "bad tensor id");
  const int64_t n = s->cfg.num_envs, np = s->S.np;
  memset(d, 0, sizeof(*d));
  d->offset_bytes = s->L.off[id];
  d->dtype = dtype_of(id);
  switch (id) {
    case HG_T_OBS_BUF:  // the history windows: [N, (F - 1 + HW) * width]; the stack = columns
    case HG_T_PRIV_BUF: {  // [head * width, (head + F) * width) (hg_obs_head)
      const int64_t w = id == HG_T_OBS_BUF ? (int64_t)win_frames(s->cfg.frame_stack, &s->cfg) * HG_OBS1
                                           : (int64_t)win_frames(s->cfg.c_frame_stack, &s->cfg) * HG_PRIV1;
      d->ndim = 2;
      d->shape[0] = n; d->shape[1] = w;
      d->strides[0] = w; d->strides[1] = 1;
      return HG_OK;
    }
    case HG_T_EP_STATS:
      d->ndim = 1; d->shape[0] = 24; d->strides[0] = 1;
      return HG_OK;
    case HG_T_EP_STATS_RING:
      d->ndim = 2; d->shape[0] = HG_EP_RING; d->shape[1] = 24; d->strides[0] = 24; d->strides[1] = 1;
      return HG_OK;
    case HG_T_CONTACT_FORCES:  // [N,13,3] (net_contact_force's shape), SoA storage
      d->ndim = 3; d->shape[0] = n; d->shape[1] = HG_NB; d->shape[2] = 3;
      d->strides[0] = 1; d->strides[1] = 3 * np; d->strides[2] = np;
      return HG_OK;
    case HG_T_RIGID_STATE:     // [N,13,13] (rigid_body_state.view(N,-1,13)'s shape), SoA storage
      d->ndim = 3; d->shape[0] = n; d->shape[1] = HG_NB; d->shape[2] = 13;
      d->strides[0] = 1; d->strides[1] = 13 * np; d->strides[2] = np;
      return HG_OK;
    case HG_T_EPISODE_SUMS:
      d->ndim = 2; d->shape[0] = HG_NUM_REWARDS; d->shape[1] = n; d->strides[0] = np; d->strides[1] = 1;
      return HG_OK;
    default: {
      const int rows = soa_rows(id);
      if (rows == 1) { d->ndim = 1; d->shape[0] = n; d->strides[0] = 1; }
      else { d->ndim = 2; d->shape[0] = n; d->shape[1] = rows; d->strides[0] = 1; d->strides[1] = np; }
      return HG_OK;
    }
  }
}

int hg_step(void* sim, const float* actions, uint64_t step_counter, void* stream) {
  Sim* s = (Sim*)sim;
  if (!s || !actions) return fail(s, HG_ERR_ARG, "null argument");
  const int rc = hg_launch_step(&s->S, &s->cfg, actions, step_counter, (hipStream_t)stream);
  if (rc != 0) return fail(s, HG_ERR_HIP, "k_step launch failed");
  return HG_OK;
}

static int do_post(Sim* s, uint64_t counter, int mode, const uint8_t* mask, void* stream) {
  const int hw = win_advance(&s->cfg);
  const int old = s->head;
  const int shift = old + 1 >= hw;  // slots old + 1 .. old + F - 1 move to 0 .. F - 2
  const int head = shift ? 0 : old + 1;
  const float inv_len_s = 1.0f / ((float)s->cfg.max_episode_length * s->cfg.dt);
  const int slot = (int)(s->post_seq % HG_EP_RING);
  const HgWindow wo = {(float*)(s->arena + s->L.obs_buf), (int64_t)win_frames(s->cfg.frame_stack, &s->cfg) * HG_OBS1,
                       HG_OBS1, s->cfg.frame_stack, head, shift ? old + 1 : -1};
  const HgWindow wp = {(float*)(s->arena + s->L.priv_buf),
                       (int64_t)win_frames(s->cfg.c_frame_stack, &s->cfg) * HG_PRIV1, HG_PRIV1, s->cfg.c_frame_stack,
                       head, shift ? old + 1 : -1};
  // a step's post launch takes the pending rollout sink (reset launches leave it pending)
  const HgSink sink = mode == 0 ? s->sink : HgSink{nullptr, nullptr, nullptr};
  if (mode == 0) s->sink = HgSink{nullptr, nullptr, nullptr};
  int rc = hg_launch_post(&s->S, &s->cfg, counter, mode, mask, (float*)(s->arena + s->L.frame_obs),
                          (float*)(s->arena + s->L.frame_priv), wo, wp, inv_len_s, slot, sink, (hipStream_t)stream);
  if (rc != 0) return fail(s, HG_ERR_HIP, "k_post launch failed");
  s->ep_slot = slot;
  s->post_seq++;
  s->head = head;
  return HG_OK;
}

int hg_obs_head(void* sim) {
  Sim* s = (Sim*)sim;
  return s ? s->head : -1;
}

int hg_obs_window_advance(void* sim) {
  Sim* s = (Sim*)sim;
  return s ? win_advance(&s->cfg) : -1;
}

int hg_ep_stats_slot(void* sim) {
  Sim* s = (Sim*)sim;
  return s ? s->ep_slot : -1;
}

int hg_set_rollout_sink(void* sim, float* rewards_out, uint8_t* dones_out, uint8_t* time_outs_out) {
  Sim* s = (Sim*)sim;
  if (!s || (!rewards_out) != (!dones_out) || (time_outs_out && !rewards_out)) return HG_ERR_ARG;
  s->sink = HgSink{rewards_out, dones_out, time_outs_out};
  return HG_OK;
}

int hg_post(void* sim, uint64_t common_step_counter, void* stream) {
  Sim* s = (Sim*)sim;
  if (!s) return HG_ERR_ARG;
  return do_post(s, common_step_counter, 0, nullptr, stream);
}

int hg_update_cfg(void* sim, const hg_cfg* cfg, void* stream) {
  Sim* s = (Sim*)sim;
  if (!s || !cfg) return HG_ERR_ARG;
  const hg_cfg& o = s->cfg;
  if (cfg->num_envs != o.num_envs || cfg->frame_stack != o.frame_stack || cfg->c_frame_stack != o.c_frame_stack ||
      cfg->decimation != o.decimation || cfg->terrain_type != o.terrain_type || cfg->hf_rows != o.hf_rows ||
      cfg->hf_cols != o.hf_cols || cfg->heightfield != o.heightfield || cfg->terrain_origins != o.terrain_origins ||
      cfg->terrain_rows != o.terrain_rows || cfg->terrain_cols != o.terrain_cols)
    return fail(s, HG_ERR_ARG, "hg_update_cfg: layout fields cannot change after hg_create");
  if (cfg->pgs_iterations < 0 || cfg->pgs_iterations > 1000 || !(cfg->sim_dt > 0.f))
    return fail(s, HG_ERR_ARG, "hg_update_cfg: bad solver parameters");
  s->cfg = *cfg;
  // the device copy is read by the env-logic launches, the host copy by K_step's launch (its
  // physics scalars go by value); the host source stays valid (it is the handle's)
  if (hipMemcpyAsync((void*)s->S.cfg, &s->cfg, sizeof(hg_cfg), hipMemcpyHostToDevice, (hipStream_t)stream) != hipSuccess)
    return fail(s, HG_ERR_HIP, "hg_update_cfg: copy failed");
  return HG_OK;
}

int hg_reset_masked(void* sim, const uint8_t* mask, uint64_t counter, void* stream) {
  Sim* s = (Sim*)sim;
  if (!s) return HG_ERR_ARG;
  return do_post(s, counter, 1, mask, stream);
}

}  // extern "C"

// ---- indexed state writes
__global__ void k_set_dof(HgState S, const int32_t* ids, int n, const float* pos, const float* vel) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int e = ids[i];
  if (e < 0 || e >= S.n) return;
  for (int j = 0; j < HG_ND; j++) {
    if (pos) S.dof_pos[j * S.np + e] = pos[(size_t)i * HG_ND + j];
    if (vel) S.dof_vel[j * S.np + e] = vel[(size_t)i * HG_ND + j];
  }
  // joint limit and friction warm starts
  for (int c = (HG_MAX_CONTACTS + HG_MAX_PAIRS) * 3; c < HG_LAMW; c++) S.lambda[c * S.np + e] = 0.f;
}
__global__ void k_set_root(HgState S, const int32_t* ids, int n, const float* root) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int e = ids[i];
  if (e < 0 || e >= S.n) return;
  for (int f = 0; f < 13; f++) S.root[f * S.np + e] = root[(size_t)i * 13 + f];
  for (int c = 0; c < (HG_MAX_CONTACTS + HG_MAX_PAIRS) * 3; c++) S.lambda[c * S.np + e] = 0.f;  // contacts
}

extern "C" int hg_set_dof_state_indexed(void* sim, const int32_t* env_ids, int n, const float* dof_pos,
                                        const float* dof_vel, void* stream) {
  Sim* s = (Sim*)sim;
  if (!s || !env_ids || n < 0) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  hipLaunchKernelGGL(k_set_dof, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, s->S, env_ids, n, dof_pos, dof_vel);
  return hipGetLastError() == hipSuccess ? HG_OK : fail(s, HG_ERR_HIP, "k_set_dof launch failed");
}

extern "C" int hg_set_root_state_indexed(void* sim, const int32_t* env_ids, int n, const float* root, void* stream) {
  Sim* s = (Sim*)sim;
  if (!s || !env_ids || !root || n < 0) return HG_ERR_ARG;
  if (n == 0) return HG_OK;
  hipLaunchKernelGGL(k_set_root, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, s->S, env_ids, n, root);
  return hipGetLastError() == hipSuccess ? HG_OK : fail(s, HG_ERR_HIP, "k_set_root launch failed");
}

// ---- measured heights: one thread per (env, point)
__global__ void k_heights(HgState S, const float* __restrict__ pts, int P, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)S.n * P) return;
  const int e = (int)(t / P), k = (int)(t % P);
  const hg_cfg* cfg = S.cfg;
  if (cfg->terrain_type == 0 || cfg->heightfield == nullptr) { out[t] = 0.f; return; }
  // quat_apply_yaw (utils/math.py:39-43): keep (z, w), normalise, rotate
  const float qz = S.root[5 * S.np + e], qw = S.root[6 * S.np + e];
  const float nrm = fmaxf(sqrtf(qz * qz + qw * qw), 1e-9f);
  const f3 p = quat_apply(0.f, 0.f, qz / nrm, qw / nrm, mk(pts[2 * k], pts[2 * k + 1], 0.f));
  const float x = p.x + S.root[0 * S.np + e] + cfg->hf_border;
  const float y = p.y + S.root[1 * S.np + e] + cfg->hf_border;
  long long px = (long long)(x / cfg->hf_horizontal_scale), py = (long long)(y / cfg->hf_horizontal_scale);
  px = px < 0 ? 0 : (px > cfg->hf_rows - 2 ? cfg->hf_rows - 2 : px);
  py = py < 0 ? 0 : (py > cfg->hf_cols - 2 ? cfg->hf_cols - 2 : py);
  const int16_t* hf = cfg->heightfield;
  const int C = cfg->hf_cols;
  int h = hf[px * C + py];
  h = min(h, (int)hf[(px + 1) * C + py]);
  h = min(h, (int)hf[px * C + py + 1]);
  out[t] = (float)h * cfg->hf_vertical_scale;
}

extern "C" int hg_measure_heights(void* sim, const float* points_xy, int num_points, float* out, void* stream) {
  Sim* s = (Sim*)sim;
  if (!s || !points_xy || !out || num_points <= 0) return HG_ERR_ARG;
  const int64_t total = (int64_t)s->S.n * num_points;
  hipLaunchKernelGGL(k_heights, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, s->S,
                     points_xy, num_points, out);
  return hipGetLastError() == hipSuccess ? HG_OK : fail(s, HG_ERR_HIP, "k_heights launch failed");
}

__global__ void k_set_root_all(HgState S, const float* root) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S.n) return;
  for (int f = 0; f < 13; f++) S.root[f * S.np + e] = root[(size_t)e * 13 + f];
  for (int c = 0; c < (HG_MAX_CONTACTS + HG_MAX_PAIRS) * 3; c++) S.lambda[c * S.np + e] = 0.f;  // contacts
}
__global__ void k_set_props(HgState S, const float* fric, const float* mass) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S.n) return;
  if (fric) S.friction[e] = fric[e];
  if (mass) S.body_mass[e] = mass[e];
}

extern "C" int hg_set_root_state(void* sim, const float* root, void* stream) {
  Sim* s = (Sim*)sim;
  if (!s || !root) return HG_ERR_ARG;
  hipLaunchKernelGGL(k_set_root_all, dim3((s->S.n + 255) / 256), dim3(256), 0, (hipStream_t)stream, s->S, root);
  return hipGetLastError() == hipSuccess ? HG_OK : fail(s, HG_ERR_HIP, "k_set_root_all launch failed");
}

extern "C" int hg_set_env_props(void* sim, const float* friction, const float* base_mass, void* stream) {
  Sim* s = (Sim*)sim;
  if (!s) return HG_ERR_ARG;
  if (!friction && !base_mass) return HG_OK;
  hipLaunchKernelGGL(k_set_props, dim3((s->S.n + 255) / 256), dim3(256), 0, (hipStream_t)stream, s->S, friction,
                     base_mass);
  return hipGetLastError() == hipSuccess ? HG_OK : fail(s, HG_ERR_HIP, "k_set_props launch failed");
}

#ifndef HG_SRC_HASH
#error "build through the Makefile: HG_SRC_HASH stamps the sources the library is built from"
#endif
extern "C" const char* hg_source_hash(void) { return HG_SRC_HASH; }
extern "C" const char* hg_version(void) { return "hg_sim 0.3 (gfx950, K_step: 32 lanes/env, LDS-resident, MFMA Delassus, register PGS)"; }
