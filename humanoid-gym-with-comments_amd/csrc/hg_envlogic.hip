// hg_envlogic.hip — K_post: post-physics env logic for every env, one lane per env, no host sync.
//
// Replaces reference humanoid/envs/custom/humanoid_env.py:
//   post_physics_step :770-809 (minus refreshes), _post_physics_step_callback :1000-1016,
//   _resample_commands :1018-1032, _push_robots :665-681, check_termination :811-816,
//   compute_reward :889-907 + the 22 _reward_* terms :1170-1437, reset_idx :1109-1163
//   (+ _reset_dofs :1034-1048, _reset_root_states :1049-1072), compute_observations :818-887,
//   _get_phase/_get_gait_phase/compute_ref_state :683-744, _get_noise_scale_vec :748-768,
//   and the obs/priv clip in step() :654-657.
// Reset is mask-based (the reference's reset_buf.nonzero() host sync :796 is gone).
// Frame stacking (deque append + stack, :880-887) is k_stack_stats below: a coalesced double-buffered
// shift of the [N, frames*width] row-major history.
#include "hg_common.h"

namespace {

constexpr float kPiF = 3.14159265358979323846f;     // float(np.pi)
constexpr float kTwoPiF = 6.28318530717958647692f;  // float(2*np.pi)

// isaacgym get_euler_xyz (components mod 2pi) followed by get_euler_xyz_tensor's
// "euler[euler > pi] -= 2pi" (humanoid_env.py:51-56)
__device__ __forceinline__ float wrap_euler(float a) {
  a = a - kTwoPiF * floorf(a / kTwoPiF);
  if (a > kPiF) a -= kTwoPiF;
  return a;
}
__device__ f3 euler_xyz(float x, float y, float z, float w) {
  float sinr = 2.0f * (w * x + y * z);
  float cosr = w * w - x * x - y * y + z * z;
  float roll = atan2f(sinr, cosr);
  float sinp = 2.0f * (w * y - z * x);
  float pitch = fabsf(sinp) >= 1.0f ? copysignf(kPiF / 2.0f, sinp) : asinf(sinp);
  float siny = 2.0f * (w * z + x * y);
  float cosy = w * w + x * x - y * y - z * z;
  float yaw = atan2f(siny, cosy);
  return mk(wrap_euler(roll), wrap_euler(pitch), wrap_euler(yaw));
}
// humanoid/utils/math.py:46-49
__device__ __forceinline__ float wrap_to_pi(float a) {
  a = a - kTwoPiF * floorf(a / kTwoPiF);
  if (a > kPiF) a -= kTwoPiF;
  return a;
}
__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

struct Gait { float sin_pos, cos_pos, stance[2]; };

// _get_phase / _get_gait_phase (humanoid_env.py:683-703)
__device__ Gait gait(const hg_cfg* cfg, int64_t ep) {
  float phase = (float)ep * cfg->dt / cfg->cycle_time;
  Gait g;
  g.sin_pos = sinf(kTwoPiF * phase);
  g.cos_pos = cosf(kTwoPiF * phase);
  g.stance[0] = g.sin_pos >= 0.f ? 1.f : 0.f;
  g.stance[1] = g.sin_pos < 0.f ? 1.f : 0.f;
  if (fabsf(g.sin_pos) < 0.1f) g.stance[0] = g.stance[1] = 1.f;
  return g;
}

// _resample_commands (humanoid_env.py:1018-1032) for one env
__device__ void resample_commands(const hg_cfg* cfg, HgState& S, int e, uint64_t step, uint32_t salt) {
  const int np = S.np;
  u4 r = rng4(cfg, e, step, salt, RNG_CMD);
  float cx = (cfg->cmd_lin_x[1] - cfg->cmd_lin_x[0]) * u01(r.x) + cfg->cmd_lin_x[0];
  float cy = (cfg->cmd_lin_y[1] - cfg->cmd_lin_y[0]) * u01(r.y) + cfg->cmd_lin_y[0];
  S.commands[0 * np + e] = cx;
  S.commands[1 * np + e] = cy;
  if (cfg->heading_command)
    S.commands[3 * np + e] = (cfg->cmd_heading[1] - cfg->cmd_heading[0]) * u01(r.z) + cfg->cmd_heading[0];
  else
    S.commands[2 * np + e] = (cfg->cmd_ang_yaw[1] - cfg->cmd_ang_yaw[0]) * u01(r.z) + cfg->cmd_ang_yaw[0];
  float keep = sqrtf(cx * cx + cy * cy) > 0.2f ? 1.f : 0.f;
  S.commands[0 * np + e] = cx * keep;
  S.commands[1 * np + e] = cy * keep;
}

// reset_idx for one env (humanoid_env.py:1109-1163); episode stats accumulate into ep_stats[24..]
__device__ void reset_env(const hg_cfg* cfg, HgState& S, int e, uint64_t step, int nrew) {
  const int np = S.np;
  // _update_terrain_curriculum (humanoid_env.py:1075-1095), before the root reset reads the
  // origin; skipped for the construction-time reset (step 0, the reference's init_done gate)
  if (cfg->curriculum && step != 0) {
    const float dx = S.root[0 * np + e] - S.env_origins[0 * np + e];
    const float dy = S.root[1 * np + e] - S.env_origins[1 * np + e];
    const float dist = sqrtf(dx * dx + dy * dy);
    const float c0 = S.commands[0 * np + e], c1 = S.commands[1 * np + e];
    const bool up = dist > cfg->terrain_env_length / 2;
    const bool down = (dist < sqrtf(c0 * c0 + c1 * c1) * cfg->max_episode_length_s * 0.5f) && !up;
    int lvl = S.terrain_level[e] + (up ? 1 : 0) - (down ? 1 : 0);
    const int maxl = cfg->terrain_rows;
    if (lvl >= maxl) {  // torch.randint_like(levels, max_terrain_level)
      lvl = min((int)(u01(rng4(cfg, e, step, 0, RNG_TERRAIN).x) * (float)maxl), maxl - 1);
    } else {
      lvl = max(lvl, 0);
    }
    S.terrain_level[e] = lvl;
    const float* o = cfg->terrain_origins + ((size_t)lvl * cfg->terrain_cols + S.terrain_type[e]) * 3;
    for (int i = 0; i < 3; i++) S.env_origins[i * np + e] = o[i];
  }
  // _reset_dofs
  for (int b = 0; b < 3; b++) {
    u4 r = rng4(cfg, e, step, b, RNG_RESET_DOF);
    uint32_t u[4] = {r.x, r.y, r.z, r.w};
    for (int i = 0; i < 4; i++) {
      int j = b * 4 + i;
      S.dof_pos[j * np + e] = cfg->default_dof_pos[j] + ((0.1f - (-0.1f)) * u01(u[i]) + (-0.1f));  // default + torch_rand_float(-0.1, 0.1)
      S.dof_vel[j * np + e] = 0.f;
    }
  }
  // _reset_root_states
  float root[13];
  for (int i = 0; i < 3; i++) root[i] = cfg->init_pos[i] + S.env_origins[i * np + e];
  for (int i = 0; i < 4; i++) root[3 + i] = cfg->init_rot[i];
  for (int i = 0; i < 3; i++) { root[7 + i] = cfg->init_lin_vel[i]; root[10 + i] = cfg->init_ang_vel[i]; }
  if (cfg->terrain_type != 0) {  // custom origins: xy within 1 m of the centre
    u4 r = rng4(cfg, e, step, 0, RNG_RESET_ROOT);
    root[0] += 2.0f * u01(r.x) - 1.0f;
    root[1] += 2.0f * u01(r.y) - 1.0f;
  }
  if (cfg->fix_base_link) {
    for (int i = 7; i < 13; i++) root[i] = 0.f;
    root[2] += 1.8f;
  }
  for (int i = 0; i < 13; i++) S.root[i * np + e] = root[i];
  for (int i = 0; i < HG_LAMW; i++) S.lambda[i * np + e] = 0.f;
  resample_commands(cfg, S, e, step, 1);
  for (int j = 0; j < HG_ND; j++) {
    S.last_last_actions[j * np + e] = 0.f;
    S.actions[j * np + e] = 0.f;
    S.last_actions[j * np + e] = 0.f;
    S.last_dof_vel[j * np + e] = 0.f;
  }
  S.feet_air_time[0 * np + e] = 0.f;
  S.feet_air_time[1 * np + e] = 0.f;
  S.ep_len[e] = 0;
  S.reset_buf[e] = 1;
  float* acc = S.ep_stats + 24;
  for (int k = 0; k < nrew; k++) {
    atomicAdd(&acc[k], S.ep_sums[k * np + e]);
    S.ep_sums[k * np + e] = 0.f;
  }
  atomicAdd(&acc[22], 1.0f);
  // refresh base quat -> projected gravity (euler is recomputed by the obs pass)
  f3 g = quat_rotate_inverse(root[3], root[4], root[5], root[6], mk(0, 0, -1));
  S.proj_gravity[0 * np + e] = g.x;
  S.proj_gravity[1 * np + e] = g.y;
  S.proj_gravity[2 * np + e] = g.z;
}

}  // namespace

// mode 0: full post_physics_step; mode 1: reset envs in `mask` (all if null) + observe
__global__ void __launch_bounds__(64) k_post(HgState S, uint64_t counter, int mode, const uint8_t* mask,
                                              float* frame_obs, float* frame_priv) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S.n) return;
  const hg_cfg* cfg = S.cfg;
  const int np = S.np;
  const int nrew = HG_NUM_REWARDS;
  float q[HG_ND], qd[HG_ND], a[HG_ND];
  bool do_reset;

  if (mode == 0) {
    int64_t ep = S.ep_len[e] + 1;
    S.ep_len[e] = ep;
    float qx = S.root[3 * np + e], qy = S.root[4 * np + e], qz = S.root[5 * np + e], qw = S.root[6 * np + e];
    f3 lv = mk(S.root[7 * np + e], S.root[8 * np + e], S.root[9 * np + e]);
    f3 av = mk(S.root[10 * np + e], S.root[11 * np + e], S.root[12 * np + e]);
    f3 blv = quat_rotate_inverse(qx, qy, qz, qw, lv);
    f3 bav = quat_rotate_inverse(qx, qy, qz, qw, av);
    f3 pg = quat_rotate_inverse(qx, qy, qz, qw, mk(0, 0, -1));
    f3 eul = euler_xyz(qx, qy, qz, qw);
    S.base_lin_vel[0 * np + e] = blv.x; S.base_lin_vel[1 * np + e] = blv.y; S.base_lin_vel[2 * np + e] = blv.z;
    S.base_ang_vel[0 * np + e] = bav.x; S.base_ang_vel[1 * np + e] = bav.y; S.base_ang_vel[2 * np + e] = bav.z;
    S.proj_gravity[0 * np + e] = pg.x; S.proj_gravity[1 * np + e] = pg.y; S.proj_gravity[2 * np + e] = pg.z;
    // ---- _post_physics_step_callback
    if (ep % cfg->resample_interval == 0) resample_commands(cfg, S, e, counter, 0);
    if (cfg->heading_command) {
      f3 fwd = quat_apply(qx, qy, qz, qw, mk(1, 0, 0));
      float heading = atan2f(fwd.y, fwd.x);
      float c2 = 0.5f * wrap_to_pi(S.commands[3 * np + e] - heading);
      S.commands[2 * np + e] = fminf(fmaxf(c2, -1.f), 1.f);
    }
    if (cfg->push_robots && (counter % (uint64_t)cfg->push_interval == 0)) {
      u4 r0 = rng4(cfg, e, counter, 0, RNG_PUSH), r1 = rng4(cfg, e, counter, 1, RNG_PUSH);
      const float mv = cfg->max_push_vel_xy, ma = cfg->max_push_ang_vel;
      float px = 2.f * mv * u01(r0.x) - mv, py = 2.f * mv * u01(r0.y) - mv;
      S.push_force[0 * np + e] = px; S.push_force[1 * np + e] = py;
      S.root[7 * np + e] = px; S.root[8 * np + e] = py;
      float t0 = 2.f * ma * u01(r0.z) - ma, t1 = 2.f * ma * u01(r0.w) - ma, t2 = 2.f * ma * u01(r1.x) - ma;
      S.push_torque[0 * np + e] = t0; S.push_torque[1 * np + e] = t1; S.push_torque[2 * np + e] = t2;
      S.root[10 * np + e] = t0; S.root[11 * np + e] = t1; S.root[12 * np + e] = t2;
    }
    // ---- check_termination
    f3 fb = mk(HG_CF(S, e, 0, 0), HG_CF(S, e, 0, 1), HG_CF(S, e, 0, 2));
    float fbn = sqrtf(dot(fb, fb));
    bool timeout = ep > (int64_t)cfg->max_episode_length;
    do_reset = (fbn > 1.0f) || timeout;
    S.time_out[e] = timeout;
    S.reset_buf[e] = do_reset;
    // ---- compute_reward
    for (int j = 0; j < HG_ND; j++) {
      q[j] = S.dof_pos[j * np + e];
      qd[j] = S.dof_vel[j * np + e];
      a[j] = S.actions[j * np + e];
    }
    Gait g = gait(cfg, ep);
    const int f0 = cfg->feet_body[0], f1 = cfg->feet_body[1];
    const int k0 = cfg->knee_body[0], k1 = cfg->knee_body[1];
    auto rig = [&](int b, int f) { return HG_RS(S, e, b, f); };
    auto cfz = [&](int b, int i) { return HG_CF(S, e, b, i); };
    bool contact[2] = {cfz(f0, 2) > 5.f, cfz(f1, 2) > 5.f};
    float term[HG_NUM_REWARDS];
    // 0 action_smoothness
    {
      float t1 = 0.f, t2 = 0.f, t3 = 0.f;
      for (int j = 0; j < HG_ND; j++) {
        float la = S.last_actions[j * np + e], lla = S.last_last_actions[j * np + e];
        float d1 = la - a[j], d2 = a[j] + lla - 2.f * la;
        t1 += d1 * d1; t2 += d2 * d2; t3 += fabsf(a[j]);
      }
      term[0] = t1 + t2 + 0.05f * t3;
    }
    // 1 base_acc
    {
      float s = 0.f;
      for (int i = 0; i < 6; i++) { float d = S.last_root_vel[i * np + e] - S.root[(7 + i) * np + e]; s += d * d; }
      term[1] = expf(-sqrtf(s) * 3.f);
    }
    // 2 base_height
    {
      float mh = (rig(f0, 2) * g.stance[0] + rig(f1, 2) * g.stance[1]) / (g.stance[0] + g.stance[1]);
      float bh = S.root[2 * np + e] - (mh - 0.05f);
      term[2] = expf(-fabsf(bh - cfg->base_height_target) * 100.f);
    }
    // 3 collision (penalised body = base)
    term[3] = fbn > 0.1f ? 1.f : 0.f;
    // 4 default_joint_pos
    {
      float dn = 0.f, d[HG_ND];
      for (int j = 0; j < HG_ND; j++) { d[j] = q[j] - cfg->default_dof_pos[j]; dn += d[j] * d[j]; }
      const int* yr = cfg->yaw_roll_idx;
      float l = sqrtf(d[yr[0]] * d[yr[0]] + d[yr[1]] * d[yr[1]]);
      float r = sqrtf(d[yr[2]] * d[yr[2]] + d[yr[3]] * d[yr[3]]);
      float y = fminf(fmaxf(l + r - 0.1f, 0.f), 50.f);
      term[4] = expf(-y * 100.f) - 0.01f * sqrtf(dn);
    }
    // 5 dof_acc, 6 dof_vel, 17 torques
    {
      float sa = 0.f, sv = 0.f, st = 0.f;
      for (int j = 0; j < HG_ND; j++) {
        float acc = (S.last_dof_vel[j * np + e] - qd[j]) / cfg->dt;
        sa += acc * acc;
        sv += qd[j] * qd[j];
        float t = S.torques[j * np + e];
        st += t * t;
      }
      term[5] = sa; term[6] = sv; term[17] = st;
    }
    // 7 feet_air_time (mutates last_contacts, feet_air_time)
    {
      float r = 0.f;
      for (int f = 0; f < 2; f++) {
        bool lc = S.last_contacts[f * np + e] != 0;
        bool filt = contact[f] || (g.stance[f] != 0.f) || lc;
        float air = S.feet_air_time[f * np + e];
        float first = (air > 0.f && filt) ? 1.f : 0.f;
        if (cfg->reward_scale[7] != 0.f) {
          S.last_contacts[f * np + e] = contact[f];
          air += cfg->dt;
          r += fminf(fmaxf(air, 0.f), 0.5f) * first;
          S.feet_air_time[f * np + e] = filt ? 0.f : air;
        }
      }
      term[7] = r;
    }
    // 8 feet_clearance (mutates feet_height, last_feet_z)
    {
      float r = 0.f;
      for (int f = 0; f < 2; f++) {
        const int fb2 = f == 0 ? f0 : f1;
        float fz = rig(fb2, 2) - 0.05f;
        float fh = S.feet_height[f * np + e] + (fz - S.last_feet_z[f * np + e]);
        float swing = 1.f - g.stance[f];
        float pos = fabsf(fh - cfg->target_feet_height) < 0.01f ? 1.f : 0.f;
        r += pos * swing;
        if (cfg->reward_scale[8] != 0.f) {
          S.last_feet_z[f * np + e] = fz;
          S.feet_height[f * np + e] = contact[f] ? 0.f : fh;
        }
      }
      term[8] = r;
    }
    // 9 feet_contact_forces, 10 feet_contact_number, 12 foot_slip
    {
      float s9 = 0.f, s10 = 0.f, s12 = 0.f;
      for (int f = 0; f < 2; f++) {
        const int fb2 = f == 0 ? f0 : f1;
        float fx = cfz(fb2, 0), fy = cfz(fb2, 1), fz = cfz(fb2, 2);
        s9 += fminf(fmaxf(sqrtf(fx * fx + fy * fy + fz * fz) - cfg->max_contact_force, 0.f), 400.f);
        s10 += ((contact[f] ? 1.f : 0.f) == g.stance[f]) ? 1.f : -0.3f;
        float wx = rig(fb2, 10), wy = rig(fb2, 11);
        s12 += contact[f] ? sqrtf(sqrtf(wx * wx + wy * wy)) : 0.f;
      }
      term[9] = s9; term[10] = s10 / 2.f; term[12] = s12;
    }
    // 11 feet_distance, 14 knee_distance
    {
      float dx = rig(f0, 0) - rig(f1, 0), dy = rig(f0, 1) - rig(f1, 1);
      float d = sqrtf(dx * dx + dy * dy);
      float dmin = fminf(fmaxf(d - cfg->min_dist, -0.5f), 0.f);
      float dmax = fminf(fmaxf(d - cfg->max_dist, 0.f), 0.5f);
      term[11] = (expf(-fabsf(dmin) * 100.f) + expf(-fabsf(dmax) * 100.f)) / 2.f;
      dx = rig(k0, 0) - rig(k1, 0); dy = rig(k0, 1) - rig(k1, 1);
      d = sqrtf(dx * dx + dy * dy);
      dmin = fminf(fmaxf(d - cfg->min_dist, -0.5f), 0.f);
      dmax = fminf(fmaxf(d - cfg->max_dist / 2.f, 0.f), 0.5f);
      term[14] = (expf(-fabsf(dmin) * 100.f) + expf(-fabsf(dmax) * 100.f)) / 2.f;
    }
    // 13 joint_pos (ref_dof_pos from the previous observation pass)
    {
      float s = 0.f;
      for (int j = 0; j < HG_ND; j++) { float d = q[j] - S.ref_dof_pos[j * np + e]; s += d * d; }
      float nrm = sqrtf(s);
      term[13] = expf(-2.f * nrm) - 0.2f * fminf(fmaxf(nrm, 0.f), 0.5f);
    }
    const float cmd0 = S.commands[0 * np + e], cmd1 = S.commands[1 * np + e], cmd2 = S.commands[2 * np + e];
    // 15 low_speed
    {
      float as = fabsf(blv.x), ac = fabsf(cmd0);
      bool low = as < 0.5f * ac, high = as > 1.2f * ac, des = !(low || high);
      bool mis = sgnf(blv.x) != sgnf(cmd0);
      float r = 0.f;
      if (low) r = -1.f;
      if (high) r = 0.f;
      if (des) r = 1.2f;
      if (mis) r = -2.f;
      term[15] = r * (fabsf(cmd0) > 0.1f ? 1.f : 0.f);
    }
    // 16 orientation
    term[16] = (expf(-(fabsf(eul.x) + fabsf(eul.y)) * 10.f) + expf(-sqrtf(pg.x * pg.x + pg.y * pg.y) * 20.f)) / 2.f;
    // 18 track_vel_hard, 19 tracking_ang_vel, 20 tracking_lin_vel, 21 vel_mismatch_exp
    {
      float ex = cmd0 - blv.x, ey = cmd1 - blv.y;
      float lin_err = sqrtf(ex * ex + ey * ey);
      float ang_err = fabsf(cmd2 - bav.z);
      term[18] = (expf(-lin_err * 10.f) + expf(-ang_err * 10.f)) / 2.f - 0.2f * (lin_err + ang_err);
      float ae = cmd2 - bav.z;
      term[19] = expf(-(ae * ae) * cfg->tracking_sigma);
      term[20] = expf(-(ex * ex + ey * ey) * cfg->tracking_sigma);
      term[21] = (expf(-(blv.z * blv.z) * 10.f) + expf(-sqrtf(bav.x * bav.x + bav.y * bav.y) * 5.f)) / 2.f;
    }
    float rew = 0.f;
    for (int k = 0; k < nrew; k++) {
      float r = term[k] * cfg->reward_scale[k];
      rew += r;
      S.ep_sums[k * np + e] += r;
    }
    if (cfg->only_positive_rewards) rew = fmaxf(rew, 0.f);
    S.rew[e] = rew;
  } else {
    do_reset = (mask == nullptr) || mask[e] != 0;
    if (!do_reset) S.reset_buf[e] = 0;
  }

  // ---- reset_idx (masked)
  if (do_reset) reset_env(cfg, S, e, counter, nrew);

  // ---- compute_observations (humanoid_env.py:818-887)
  {
    int64_t ep = S.ep_len[e];
    Gait g = gait(cfg, ep);
    float qx = S.root[3 * np + e], qy = S.root[4 * np + e], qz = S.root[5 * np + e], qw = S.root[6 * np + e];
    f3 eul = euler_xyz(qx, qy, qz, qw);
    S.base_euler[0 * np + e] = eul.x; S.base_euler[1 * np + e] = eul.y; S.base_euler[2 * np + e] = eul.z;
    // compute_ref_state
    float ref[HG_ND];
    for (int j = 0; j < HG_ND; j++) ref[j] = 0.f;
    const float sl = fminf(g.sin_pos, 0.f), sr = fmaxf(g.sin_pos, 0.f);
    const float s1 = cfg->target_joint_pos_scale, s2 = 2.f * s1;
    const int* ri = cfg->ref_idx;
    ref[ri[0]] = sl * s1; ref[ri[1]] = sl * s2; ref[ri[2]] = sl * s1;
    ref[ri[3]] = sr * s1; ref[ri[4]] = sr * s2; ref[ri[5]] = sr * s1;
    if (fabsf(g.sin_pos) < 0.1f)
      for (int j = 0; j < HG_ND; j++) ref[j] = 0.f;
    for (int j = 0; j < HG_ND; j++) S.ref_dof_pos[j * np + e] = ref[j];
    const int f0 = cfg->feet_body[0], f1 = cfg->feet_body[1];
    float cm0 = HG_CF(S, e, f0, 2) > 5.f ? 1.f : 0.f;
    float cm1 = HG_CF(S, e, f1, 2) > 5.f ? 1.f : 0.f;
    float c0 = S.commands[0 * np + e] * cfg->obs_lin_vel, c1 = S.commands[1 * np + e] * cfg->obs_lin_vel;
    float c2 = S.commands[2 * np + e] * cfg->obs_ang_vel;
    float* P = frame_priv + (size_t)e * HG_PRIV1;
    float* O = frame_obs + (size_t)e * HG_OBS1;
    const float clip = cfg->clip_observations;
    auto cl = [clip](float v) { return fminf(fmaxf(v, -clip), clip); };
    // privileged frame (73)
    P[0] = cl(g.sin_pos); P[1] = cl(g.cos_pos); P[2] = cl(c0); P[3] = cl(c1); P[4] = cl(c2);
    for (int j = 0; j < HG_ND; j++) {
      float qj = S.dof_pos[j * np + e], qdj = S.dof_vel[j * np + e], aj = S.actions[j * np + e];
      P[5 + j] = cl((qj - cfg->default_dof_pos[j]) * cfg->obs_dof_pos);
      P[17 + j] = cl(qdj * cfg->obs_dof_vel);
      P[29 + j] = cl(aj);
      P[41 + j] = cl(qj - ref[j]);
    }
    f3 blv = mk(S.base_lin_vel[0 * np + e], S.base_lin_vel[1 * np + e], S.base_lin_vel[2 * np + e]);
    f3 bav = mk(S.base_ang_vel[0 * np + e], S.base_ang_vel[1 * np + e], S.base_ang_vel[2 * np + e]);
    P[53] = cl(blv.x * cfg->obs_lin_vel); P[54] = cl(blv.y * cfg->obs_lin_vel); P[55] = cl(blv.z * cfg->obs_lin_vel);
    P[56] = cl(bav.x * cfg->obs_ang_vel); P[57] = cl(bav.y * cfg->obs_ang_vel); P[58] = cl(bav.z * cfg->obs_ang_vel);
    P[59] = cl(eul.x * cfg->obs_quat); P[60] = cl(eul.y * cfg->obs_quat); P[61] = cl(eul.z * cfg->obs_quat);
    P[62] = cl(S.push_force[0 * np + e]); P[63] = cl(S.push_force[1 * np + e]);
    P[64] = cl(S.push_torque[0 * np + e]); P[65] = cl(S.push_torque[1 * np + e]); P[66] = cl(S.push_torque[2 * np + e]);
    P[67] = cl(S.friction[e]);
    P[68] = cl(S.body_mass[e] / 30.f);
    P[69] = g.stance[0]; P[70] = g.stance[1];
    P[71] = cm0; P[72] = cm1;
    // observation frame (47) + noise
    float z[48];
    if (cfg->add_noise) {
      for (int b = 0; b < 12; b++) normals4(rng4(cfg, e, counter, b, RNG_OBS_NOISE), z + 4 * b);
    } else {
      for (int i = 0; i < 48; i++) z[i] = 0.f;
    }
    const float nl = cfg->noise_level;
    O[0] = cl(g.sin_pos); O[1] = cl(g.cos_pos); O[2] = cl(c0); O[3] = cl(c1); O[4] = cl(c2);
    for (int j = 0; j < HG_ND; j++) {
      float qj = S.dof_pos[j * np + e], qdj = S.dof_vel[j * np + e], aj = S.actions[j * np + e];
      O[5 + j] = cl((qj - cfg->default_dof_pos[j]) * cfg->obs_dof_pos + z[5 + j] * (cfg->noise_dof_pos * cfg->obs_dof_pos) * nl);
      O[17 + j] = cl(qdj * cfg->obs_dof_vel + z[17 + j] * (cfg->noise_dof_vel * cfg->obs_dof_vel) * nl);
      O[29 + j] = cl(aj);
    }
    O[41] = cl(bav.x * cfg->obs_ang_vel + z[41] * (cfg->noise_ang_vel * cfg->obs_ang_vel) * nl);
    O[42] = cl(bav.y * cfg->obs_ang_vel + z[42] * (cfg->noise_ang_vel * cfg->obs_ang_vel) * nl);
    O[43] = cl(bav.z * cfg->obs_ang_vel + z[43] * (cfg->noise_ang_vel * cfg->obs_ang_vel) * nl);
    O[44] = cl(eul.x * cfg->obs_quat + z[44] * (cfg->noise_quat * cfg->obs_quat) * nl);
    O[45] = cl(eul.y * cfg->obs_quat + z[45] * (cfg->noise_quat * cfg->obs_quat) * nl);
    O[46] = cl(eul.z * cfg->obs_quat + z[46] * (cfg->noise_quat * cfg->obs_quat) * nl);
  }
  // ---- last_* copies (post_physics_step :802-806)
  if (mode == 0) {
    for (int j = 0; j < HG_ND; j++) {
      S.last_last_actions[j * np + e] = S.last_actions[j * np + e];
      S.last_actions[j * np + e] = S.actions[j * np + e];
      S.last_dof_vel[j * np + e] = S.dof_vel[j * np + e];
    }
    for (int i = 0; i < 6; i++) S.last_root_vel[i * np + e] = S.root[(7 + i) * np + e];
  }
}

// K_post for a policy step (mode 0 of k_post, same arithmetic in the same order), restructured for
// latency: one lane per env and 64 envs per block leave one wave per CU, so the kernel time is
// the number of dependent memory round trips.  Every per-env input is loaded up front (no store
// precedes a load, so the loads issue back to back), the step is computed in registers, the
// outputs are stored once; cfg is a by-value kernel argument (scalar loads).  The rare reset
// branch goes through reset_env and reloads the state it rewrote.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) k_post_step(HgState S, const hg_cfg C, uint64_t counter,
                                                   float* __restrict__ frame_obs, float* __restrict__ frame_priv) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S.n) return;
  const hg_cfg* cfg = &C;
  const int np = S.np;
  const int f0 = C.feet_body[0], f1 = C.feet_body[1];
  const int k0 = C.knee_body[0], k1 = C.knee_body[1];
  // ---------------- loads
  float root[13], q[HG_ND], qd[HG_ND], a[HG_ND], la[HG_ND], lla[HG_ND], ldv[HG_ND], tq[HG_ND], refp[HG_ND];
  float lrv[6], cmd[4], es[HG_NUM_REWARDS];
#pragma unroll
  for (int i = 0; i < 13; i++) root[i] = S.root[i * np + e];
#pragma unroll
  for (int j = 0; j < HG_ND; j++) {
    q[j] = S.dof_pos[j * np + e];
    qd[j] = S.dof_vel[j * np + e];
    a[j] = S.actions[j * np + e];
    la[j] = S.last_actions[j * np + e];
    lla[j] = S.last_last_actions[j * np + e];
    ldv[j] = S.last_dof_vel[j * np + e];
    tq[j] = S.torques[j * np + e];
    refp[j] = S.ref_dof_pos[j * np + e];
  }
#pragma unroll
  for (int i = 0; i < 6; i++) lrv[i] = S.last_root_vel[i * np + e];
#pragma unroll
  for (int i = 0; i < 4; i++) cmd[i] = S.commands[i * np + e];
#pragma unroll
  for (int k = 0; k < HG_NUM_REWARDS; k++) es[k] = S.ep_sums[k * np + e];
  int64_t ep = S.ep_len[e] + 1;
  const float cb0 = HG_CF(S, e, 0, 0), cb1 = HG_CF(S, e, 0, 1), cb2 = HG_CF(S, e, 0, 2);
  const float cf0x = HG_CF(S, e, f0, 0), cf0y = HG_CF(S, e, f0, 1), cf0z = HG_CF(S, e, f0, 2);
  const float cf1x = HG_CF(S, e, f1, 0), cf1y = HG_CF(S, e, f1, 1), cf1z = HG_CF(S, e, f1, 2);
  const float r0x = HG_RS(S, e, f0, 0), r0y = HG_RS(S, e, f0, 1), r0z = HG_RS(S, e, f0, 2);
  const float r0wx = HG_RS(S, e, f0, 10), r0wy = HG_RS(S, e, f0, 11);
  const float r1x = HG_RS(S, e, f1, 0), r1y = HG_RS(S, e, f1, 1), r1z = HG_RS(S, e, f1, 2);
  const float r1wx = HG_RS(S, e, f1, 10), r1wy = HG_RS(S, e, f1, 11);
  const float kn0x = HG_RS(S, e, k0, 0), kn0y = HG_RS(S, e, k0, 1);
  const float kn1x = HG_RS(S, e, k1, 0), kn1y = HG_RS(S, e, k1, 1);
  float fat[2] = {S.feet_air_time[e], S.feet_air_time[np + e]};
  bool lc[2] = {S.last_contacts[e] != 0, S.last_contacts[np + e] != 0};
  float fht[2] = {S.feet_height[e], S.feet_height[np + e]};
  float lfz[2] = {S.last_feet_z[e], S.last_feet_z[np + e]};
  float pf[3] = {S.push_force[e], S.push_force[np + e], S.push_force[2 * np + e]};
  float pt[3] = {S.push_torque[e], S.push_torque[np + e], S.push_torque[2 * np + e]};
  const float fric = S.friction[e], bmass = S.body_mass[e];

  // ---------------- post_physics_step (k_post mode 0, same expressions)
  const float qx = root[3], qy = root[4], qz = root[5], qw = root[6];
  const f3 blv = quat_rotate_inverse(qx, qy, qz, qw, mk(root[7], root[8], root[9]));
  const f3 bav = quat_rotate_inverse(qx, qy, qz, qw, mk(root[10], root[11], root[12]));
  const f3 pg = quat_rotate_inverse(qx, qy, qz, qw, mk(0, 0, -1));
  const f3 eul = euler_xyz(qx, qy, qz, qw);
  if (ep % C.resample_interval == 0) {  // resample_commands
    u4 r = rng4(cfg, e, counter, 0, RNG_CMD);
    float cx = (C.cmd_lin_x[1] - C.cmd_lin_x[0]) * u01(r.x) + C.cmd_lin_x[0];
    float cy = (C.cmd_lin_y[1] - C.cmd_lin_y[0]) * u01(r.y) + C.cmd_lin_y[0];
    if (C.heading_command) cmd[3] = (C.cmd_heading[1] - C.cmd_heading[0]) * u01(r.z) + C.cmd_heading[0];
    else cmd[2] = (C.cmd_ang_yaw[1] - C.cmd_ang_yaw[0]) * u01(r.z) + C.cmd_ang_yaw[0];
    float keep = sqrtf(cx * cx + cy * cy) > 0.2f ? 1.f : 0.f;
    cmd[0] = cx * keep;
    cmd[1] = cy * keep;
  }
  if (C.heading_command) {
    f3 fwd = quat_apply(qx, qy, qz, qw, mk(1, 0, 0));
    float heading = atan2f(fwd.y, fwd.x);
    float c2 = 0.5f * wrap_to_pi(cmd[3] - heading);
    cmd[2] = fminf(fmaxf(c2, -1.f), 1.f);
  }
  const bool pushed = C.push_robots && (counter % (uint64_t)C.push_interval == 0);
  if (pushed) {
    u4 p0 = rng4(cfg, e, counter, 0, RNG_PUSH), p1 = rng4(cfg, e, counter, 1, RNG_PUSH);
    const float mv = C.max_push_vel_xy, ma = C.max_push_ang_vel;
    float px = 2.f * mv * u01(p0.x) - mv, py = 2.f * mv * u01(p0.y) - mv;
    pf[0] = px; pf[1] = py;
    root[7] = px; root[8] = py;
    float t0 = 2.f * ma * u01(p0.z) - ma, t1 = 2.f * ma * u01(p0.w) - ma, t2 = 2.f * ma * u01(p1.x) - ma;
    pt[0] = t0; pt[1] = t1; pt[2] = t2;
    root[10] = t0; root[11] = t1; root[12] = t2;
  }
  const float fbn = sqrtf(cb0 * cb0 + cb1 * cb1 + cb2 * cb2);
  const bool timeout = ep > (int64_t)C.max_episode_length;
  const bool do_reset = (fbn > 1.0f) || timeout;
  // compute_reward
  Gait g = gait(cfg, ep);
  const bool contact[2] = {cf0z > 5.f, cf1z > 5.f};
  float term[HG_NUM_REWARDS];
  {  // 0 action_smoothness
    float t1 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
    for (int j = 0; j < HG_ND; j++) {
      float d1 = la[j] - a[j], d2 = a[j] + lla[j] - 2.f * la[j];
      t1 += d1 * d1; t2 += d2 * d2; t3 += fabsf(a[j]);
    }
    term[0] = t1 + t2 + 0.05f * t3;
  }
  {  // 1 base_acc
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 6; i++) { float d = lrv[i] - root[7 + i]; s += d * d; }
    term[1] = expf(-sqrtf(s) * 3.f);
  }
  {  // 2 base_height
    float mh = (r0z * g.stance[0] + r1z * g.stance[1]) / (g.stance[0] + g.stance[1]);
    float bh = root[2] - (mh - 0.05f);
    term[2] = expf(-fabsf(bh - C.base_height_target) * 100.f);
  }
  term[3] = fbn > 0.1f ? 1.f : 0.f;  // 3 collision
  {  // 4 default_joint_pos
    float dn = 0.f, d[HG_ND];
#pragma unroll
    for (int j = 0; j < HG_ND; j++) { d[j] = q[j] - C.default_dof_pos[j]; dn += d[j] * d[j]; }
    float dy[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < HG_ND; j++) v = (j == C.yaw_roll_idx[m]) ? d[j] : v;
      dy[m] = v;
    }
    float l = sqrtf(dy[0] * dy[0] + dy[1] * dy[1]);
    float r = sqrtf(dy[2] * dy[2] + dy[3] * dy[3]);
    float y = fminf(fmaxf(l + r - 0.1f, 0.f), 50.f);
    term[4] = expf(-y * 100.f) - 0.01f * sqrtf(dn);
  }
  {  // 5 dof_acc, 6 dof_vel, 17 torques
    float sa = 0.f, sv = 0.f, st = 0.f;
#pragma unroll
    for (int j = 0; j < HG_ND; j++) {
      float acc = (ldv[j] - qd[j]) / C.dt;
      sa += acc * acc;
      sv += qd[j] * qd[j];
      st += tq[j] * tq[j];
    }
    term[5] = sa; term[6] = sv; term[17] = st;
  }
  {  // 7 feet_air_time
    float r = 0.f;
#pragma unroll
    for (int f = 0; f < 2; f++) {
      bool filt = contact[f] || (g.stance[f] != 0.f) || lc[f];
      float air = fat[f];
      float first = (air > 0.f && filt) ? 1.f : 0.f;
      if (C.reward_scale[7] != 0.f) {
        lc[f] = contact[f];
        air += C.dt;
        r += fminf(fmaxf(air, 0.f), 0.5f) * first;
        fat[f] = filt ? 0.f : air;
      }
    }
    term[7] = r;
  }
  {  // 8 feet_clearance
    float r = 0.f;
#pragma unroll
    for (int f = 0; f < 2; f++) {
      float fz = (f == 0 ? r0z : r1z) - 0.05f;
      float fh = fht[f] + (fz - lfz[f]);
      float swing = 1.f - g.stance[f];
      float pos = fabsf(fh - C.target_feet_height) < 0.01f ? 1.f : 0.f;
      r += pos * swing;
      if (C.reward_scale[8] != 0.f) {
        lfz[f] = fz;
        fht[f] = contact[f] ? 0.f : fh;
      }
    }
    term[8] = r;
  }
  {  // 9 feet_contact_forces, 10 feet_contact_number, 12 foot_slip
    float s9 = 0.f, s10 = 0.f, s12 = 0.f;
#pragma unroll
    for (int f = 0; f < 2; f++) {
      float fx = f == 0 ? cf0x : cf1x, fy = f == 0 ? cf0y : cf1y, fz = f == 0 ? cf0z : cf1z;
      s9 += fminf(fmaxf(sqrtf(fx * fx + fy * fy + fz * fz) - C.max_contact_force, 0.f), 400.f);
      s10 += ((contact[f] ? 1.f : 0.f) == g.stance[f]) ? 1.f : -0.3f;
      float wx = f == 0 ? r0wx : r1wx, wy = f == 0 ? r0wy : r1wy;
      s12 += contact[f] ? sqrtf(sqrtf(wx * wx + wy * wy)) : 0.f;
    }
    term[9] = s9; term[10] = s10 / 2.f; term[12] = s12;
  }
  {  // 11 feet_distance, 14 knee_distance
    float dx = r0x - r1x, dy = r0y - r1y;
    float d = sqrtf(dx * dx + dy * dy);
    float dmin = fminf(fmaxf(d - C.min_dist, -0.5f), 0.f);
    float dmax = fminf(fmaxf(d - C.max_dist, 0.f), 0.5f);
    term[11] = (expf(-fabsf(dmin) * 100.f) + expf(-fabsf(dmax) * 100.f)) / 2.f;
    dx = kn0x - kn1x; dy = kn0y - kn1y;
    d = sqrtf(dx * dx + dy * dy);
    dmin = fminf(fmaxf(d - C.min_dist, -0.5f), 0.f);
    dmax = fminf(fmaxf(d - C.max_dist / 2.f, 0.f), 0.5f);
    term[14] = (expf(-fabsf(dmin) * 100.f) + expf(-fabsf(dmax) * 100.f)) / 2.f;
  }
  {  // 13 joint_pos (ref_dof_pos from the previous observation pass)
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < HG_ND; j++) { float d = q[j] - refp[j]; s += d * d; }
    float nrm = sqrtf(s);
    term[13] = expf(-2.f * nrm) - 0.2f * fminf(fmaxf(nrm, 0.f), 0.5f);
  }
  const float cmd0 = cmd[0], cmd1 = cmd[1], cmd2 = cmd[2];
  {  // 15 low_speed
    float as = fabsf(blv.x), ac = fabsf(cmd0);
    bool low = as < 0.5f * ac, high = as > 1.2f * ac, des = !(low || high);
    bool mis = sgnf(blv.x) != sgnf(cmd0);
    float r = 0.f;
    if (low) r = -1.f;
    if (high) r = 0.f;
    if (des) r = 1.2f;
    if (mis) r = -2.f;
    term[15] = r * (fabsf(cmd0) > 0.1f ? 1.f : 0.f);
  }
  term[16] = (expf(-(fabsf(eul.x) + fabsf(eul.y)) * 10.f) + expf(-sqrtf(pg.x * pg.x + pg.y * pg.y) * 20.f)) / 2.f;
  {  // 18 track_vel_hard, 19 tracking_ang_vel, 20 tracking_lin_vel, 21 vel_mismatch_exp
    float ex = cmd0 - blv.x, ey = cmd1 - blv.y;
    float lin_err = sqrtf(ex * ex + ey * ey);
    float ang_err = fabsf(cmd2 - bav.z);
    term[18] = (expf(-lin_err * 10.f) + expf(-ang_err * 10.f)) / 2.f - 0.2f * (lin_err + ang_err);
    float ae = cmd2 - bav.z;
    term[19] = expf(-(ae * ae) * C.tracking_sigma);
    term[20] = expf(-(ex * ex + ey * ey) * C.tracking_sigma);
    term[21] = (expf(-(blv.z * blv.z) * 10.f) + expf(-sqrtf(bav.x * bav.x + bav.y * bav.y) * 5.f)) / 2.f;
  }
  float rew = 0.f;
#pragma unroll
  for (int k = 0; k < HG_NUM_REWARDS; k++) {
    float r = term[k] * C.reward_scale[k];
    rew += r;
    es[k] += r;
  }
  if (C.only_positive_rewards) rew = fmaxf(rew, 0.f);

  // ---------------- stores of the step's state
  S.ep_len[e] = ep;
  S.base_lin_vel[e] = blv.x; S.base_lin_vel[np + e] = blv.y; S.base_lin_vel[2 * np + e] = blv.z;
  S.base_ang_vel[e] = bav.x; S.base_ang_vel[np + e] = bav.y; S.base_ang_vel[2 * np + e] = bav.z;
  S.proj_gravity[e] = pg.x; S.proj_gravity[np + e] = pg.y; S.proj_gravity[2 * np + e] = pg.z;
#pragma unroll
  for (int i = 0; i < 4; i++) S.commands[i * np + e] = cmd[i];
  if (pushed) {
    S.push_force[e] = pf[0]; S.push_force[np + e] = pf[1];
    S.root[7 * np + e] = root[7]; S.root[8 * np + e] = root[8];
    S.push_torque[e] = pt[0]; S.push_torque[np + e] = pt[1]; S.push_torque[2 * np + e] = pt[2];
    S.root[10 * np + e] = root[10]; S.root[11 * np + e] = root[11]; S.root[12 * np + e] = root[12];
  }
  S.time_out[e] = timeout;
  S.reset_buf[e] = do_reset;
  S.last_contacts[e] = lc[0]; S.last_contacts[np + e] = lc[1];
  S.feet_air_time[e] = fat[0]; S.feet_air_time[np + e] = fat[1];
  S.last_feet_z[e] = lfz[0]; S.last_feet_z[np + e] = lfz[1];
  S.feet_height[e] = fht[0]; S.feet_height[np + e] = fht[1];
#pragma unroll
  for (int k = 0; k < HG_NUM_REWARDS; k++) S.ep_sums[k * np + e] = es[k];
  S.rew[e] = rew;

  // ---------------- reset_idx (rare): reset_env rewrites the state in memory; reload what the
  // observation and the last_* copies read
  if (do_reset) {
    reset_env(cfg, S, e, counter, HG_NUM_REWARDS);
    ep = 0;
#pragma unroll
    for (int i = 0; i < 13; i++) root[i] = S.root[i * np + e];
#pragma unroll
    for (int j = 0; j < HG_ND; j++) {
      q[j] = S.dof_pos[j * np + e];
      qd[j] = S.dof_vel[j * np + e];
      a[j] = 0.f;
      la[j] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) cmd[i] = S.commands[i * np + e];
  }

  // ---------------- compute_observations (humanoid_env.py:818-887), as k_post
  {
    Gait go = gait(cfg, ep);
    const f3 eo = euler_xyz(root[3], root[4], root[5], root[6]);
    S.base_euler[e] = eo.x; S.base_euler[np + e] = eo.y; S.base_euler[2 * np + e] = eo.z;
    float ref[HG_ND];
    const float sl = fminf(go.sin_pos, 0.f), sr = fmaxf(go.sin_pos, 0.f);
    const float s1 = C.target_joint_pos_scale, s2 = 2.f * s1;
    const bool zero = fabsf(go.sin_pos) < 0.1f;
#pragma unroll
    for (int j = 0; j < HG_ND; j++) {
      // the later assignment wins when indices coincide, as in k_post's sequential stores
      float v = 0.f;
      v = (j == C.ref_idx[0]) ? sl * s1 : v;
      v = (j == C.ref_idx[1]) ? sl * s2 : v;
      v = (j == C.ref_idx[2]) ? sl * s1 : v;
      v = (j == C.ref_idx[3]) ? sr * s1 : v;
      v = (j == C.ref_idx[4]) ? sr * s2 : v;
      v = (j == C.ref_idx[5]) ? sr * s1 : v;
      ref[j] = zero ? 0.f : v;
      S.ref_dof_pos[j * np + e] = ref[j];
    }
    const float cm0 = cf0z > 5.f ? 1.f : 0.f;
    const float cm1 = cf1z > 5.f ? 1.f : 0.f;
    const float c0 = cmd[0] * C.obs_lin_vel, c1 = cmd[1] * C.obs_lin_vel;
    const float c2 = cmd[2] * C.obs_ang_vel;
    float* P = frame_priv + (size_t)e * HG_PRIV1;
    float* O = frame_obs + (size_t)e * HG_OBS1;
    const float clip = C.clip_observations;
    auto cl = [clip](float v) { return fminf(fmaxf(v, -clip), clip); };
    P[0] = cl(go.sin_pos); P[1] = cl(go.cos_pos); P[2] = cl(c0); P[3] = cl(c1); P[4] = cl(c2);
#pragma unroll
    for (int j = 0; j < HG_ND; j++) {
      P[5 + j] = cl((q[j] - C.default_dof_pos[j]) * C.obs_dof_pos);
      P[17 + j] = cl(qd[j] * C.obs_dof_vel);
      P[29 + j] = cl(a[j]);
      P[41 + j] = cl(q[j] - ref[j]);
    }
    P[53] = cl(blv.x * C.obs_lin_vel); P[54] = cl(blv.y * C.obs_lin_vel); P[55] = cl(blv.z * C.obs_lin_vel);
    P[56] = cl(bav.x * C.obs_ang_vel); P[57] = cl(bav.y * C.obs_ang_vel); P[58] = cl(bav.z * C.obs_ang_vel);
    P[59] = cl(eo.x * C.obs_quat); P[60] = cl(eo.y * C.obs_quat); P[61] = cl(eo.z * C.obs_quat);
    P[62] = cl(pf[0]); P[63] = cl(pf[1]);
    P[64] = cl(pt[0]); P[65] = cl(pt[1]); P[66] = cl(pt[2]);
    P[67] = cl(fric);
    P[68] = cl(bmass / 30.f);
    P[69] = go.stance[0]; P[70] = go.stance[1];
    P[71] = cm0; P[72] = cm1;
    float z[48];
    if (C.add_noise && *S.noise_counter == counter) {
      // drawn by the K_step epilogue for this counter (same Philox keys, same values)
      const float4* zr = reinterpret_cast<const float4*>(S.obs_noise + (size_t)e * 48);
#pragma unroll
      for (int q = 0; q < 12; q++) {
        const float4 v = zr[q];
        z[4 * q] = v.x; z[4 * q + 1] = v.y; z[4 * q + 2] = v.z; z[4 * q + 3] = v.w;
      }
    } else if (C.add_noise) {
#pragma unroll
      for (int b = 0; b < 12; b++) normals4(rng4(cfg, e, counter, b, RNG_OBS_NOISE), z + 4 * b);
    } else {
#pragma unroll
      for (int i = 0; i < 48; i++) z[i] = 0.f;
    }
    const float nl = C.noise_level;
    O[0] = cl(go.sin_pos); O[1] = cl(go.cos_pos); O[2] = cl(c0); O[3] = cl(c1); O[4] = cl(c2);
#pragma unroll
    for (int j = 0; j < HG_ND; j++) {
      O[5 + j] = cl((q[j] - C.default_dof_pos[j]) * C.obs_dof_pos + z[5 + j] * (C.noise_dof_pos * C.obs_dof_pos) * nl);
      O[17 + j] = cl(qd[j] * C.obs_dof_vel + z[17 + j] * (C.noise_dof_vel * C.obs_dof_vel) * nl);
      O[29 + j] = cl(a[j]);
    }
    O[41] = cl(bav.x * C.obs_ang_vel + z[41] * (C.noise_ang_vel * C.obs_ang_vel) * nl);
    O[42] = cl(bav.y * C.obs_ang_vel + z[42] * (C.noise_ang_vel * C.obs_ang_vel) * nl);
    O[43] = cl(bav.z * C.obs_ang_vel + z[43] * (C.noise_ang_vel * C.obs_ang_vel) * nl);
    O[44] = cl(eo.x * C.obs_quat + z[44] * (C.noise_quat * C.obs_quat) * nl);
    O[45] = cl(eo.y * C.obs_quat + z[45] * (C.noise_quat * C.obs_quat) * nl);
    O[46] = cl(eo.z * C.obs_quat + z[46] * (C.noise_quat * C.obs_quat) * nl);
  }
  // ---------------- last_* copies (post_physics_step :802-806)
#pragma unroll
  for (int j = 0; j < HG_ND; j++) {
    S.last_last_actions[j * np + e] = la[j];
    S.last_actions[j * np + e] = a[j];
    S.last_dof_vel[j * np + e] = qd[j];
  }
#pragma unroll
  for (int i = 0; i < 6; i++) S.last_root_vel[i * np + e] = root[7 + i];
}

// history stacking: dst[e] = [src[e][W:], frame[e]] (src zeroed for reset envs), for the
// observation and the privileged tables in one launch; one block per (env, table) row, threads
// along the row so both the reads and the writes are contiguous.  The last block also folds the episode statistics
// (ep_stats[k] = acc[k] / n_reset / episode_length_s when any env reset) and clears the
// accumulators.
struct StackT {
  const float* src;
  float* dst;
  const float* frame;
  int width, frames;
};
__global__ void __launch_bounds__(256) k_stack_stats(StackT A, StackT B, const uint8_t* __restrict__ reset, int n,
                                                     float* ep_stats, float inv_len_s, int ring_slot) {
  if (blockIdx.x == gridDim.x - 1) {
    const int k = threadIdx.x;
    float* acc = ep_stats + 24;
    const float cnt = acc[22];
    __syncthreads();
    float v = k < 24 ? ep_stats[k] : 0.f;
    if (k < HG_NUM_REWARDS && cnt > 0.f) v = acc[k] / cnt * inv_len_s;
    if (k == 22) v = cnt;
    if (k == 23) v = cnt > 0.f ? 1.f : 0.f;
    if (k < 24) {
      ep_stats[k] = v;
      ep_stats[48 + ring_slot * 24 + k] = v;  // this launch's snapshot (HG_T_EP_STATS_RING)
    }
    __syncthreads();
    if (k < 24) acc[k] = 0.f;
    return;
  }
  // one block per (env, table) row: no per-element index division (the former flat one-thread-
  // per-element form spent its time in 64-bit divides), contiguous reads and writes along the row
  const int b = blockIdx.x;
  const bool a = b < n;
  const StackT& T = a ? A : B;
  const int e = a ? b : b - n;
  const int row = T.frames * T.width;
  const int cut = row - T.width;
  const bool rs = reset[e] != 0;
  const float* __restrict__ src = T.src + (size_t)e * row + T.width;
  const float* __restrict__ fr = T.frame + (size_t)e * T.width - cut;
  float* __restrict__ dst = T.dst + (size_t)e * row;
  for (int k = threadIdx.x; k < row; k += blockDim.x) dst[k] = k >= cut ? fr[k] : (rs ? 0.f : src[k]);
}

extern "C" int hg_launch_post(const HgState* S, const hg_cfg* hcfg, uint64_t counter, int mode, const uint8_t* mask,
                              float* frame_obs, float* frame_priv, const float* obs_src, float* obs_dst,
                              const float* priv_src, float* priv_dst, int frame_stack, int c_frame_stack,
                              float inv_len_s, int ep_slot, hipStream_t stream) {
  const int n = S->n;
  if (mode == 0)
    hipLaunchKernelGGL(k_post_step, dim3((n + 63) / 64), dim3(64), 0, stream, *S, *hcfg, counter, frame_obs,
                       frame_priv);
  else
    hipLaunchKernelGGL(k_post, dim3((n + 63) / 64), dim3(64), 0, stream, *S, counter, mode, mask, frame_obs,
                       frame_priv);
  const int g = 2 * n + 1;  // one block per (env, table) row + the statistics block
  const StackT A = {obs_src, obs_dst, frame_obs, HG_OBS1, frame_stack};
  const StackT B = {priv_src, priv_dst, frame_priv, HG_PRIV1, c_frame_stack};
  hipLaunchKernelGGL(k_stack_stats, dim3(g), dim3(256), 0, stream, A, B, S->reset_buf, n, S->ep_stats, inv_len_s,
                     ep_slot);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
