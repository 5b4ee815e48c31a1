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
// Frame stacking (deque append + stack, :880-887) is k_window_stats below: one frame written per env
// into a sliding history window (no copy of the whole stack).
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
  sincosf(kTwoPiF * phase, &g.sin_pos, &g.cos_pos);  // one argument reduction for both
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

#ifndef HG_POST_PEB
#define HG_POST_PEB 16
#endif
// K_post for a policy step (mode 0 of k_post, same arithmetic in the same order; exponentials by
// the hardware exp, __expf, within the reward tolerance).
//
// One lane per env, eight waves per block, and every wave a different job over the block's 64 envs:
// the post-physics chain is a long scalar dependency chain per env, so its latency is the
// instruction count one wave issues; eight waves with eight slices of it (wave-uniform code, no
// divergence) finish in about an eighth of the time one lane per env took.  Phases, separated by
// LDS-only barriers (each global location has one writer per env, so no phase waits for another's
// stores):
//   L  the block's 64-env slice of every SoA input row staged into LDS (slot-major [slot][64]),
//      each wave loading a fixed set of rows, all loads issued before the first LDS write;
//   D  derived state: base frame velocities / gravity + termination, euler angles, commands,
//      gait phase, push, and the joint sums (three waves);
//   T  the 22 reward terms, ~3 per wave, with the feet state updates; reward = sum of the waves'
//      partial sums;
//   R  reset_idx for the resetting lanes, split by field (root + curriculum, joints, lambda rows,
//      commands, episode statistics, counters); the new state goes straight into LDS;
//   O  observation / privileged frames built in LDS by joint and field groups, then written out
//      row-major with coalesced float4 stores; the last_* copies.
namespace {
constexpr int PEB = HG_POST_PEB;  // envs per block: lanes 0..PEB-1 of every wave, one env each
static_assert(PEB == 16 || PEB == 32 || PEB == 64, "envs per block");
constexpr int PWAVES = 8;   // waves per block
// LDS slots ([slot][64] floats; ints stored through their bit patterns)
enum PostSlot {
  // inputs
  X_ROOT = 0, X_CMD = 13, X_LRV = 17, X_FAT = 23, X_FHT = 25, X_LFZ = 27, X_PF = 29, X_PT = 32, X_FRIC = 35,
  X_BMASS = 36, X_ES = 37, X_CF = 59 /* base xyz, foot0 xyz, foot1 xyz */,
  X_RG = 68 /* foot0 x y z wx wy, foot1 x y z wx wy, knee0 x y, knee1 x y */, X_LC = 82, X_EP = 84, X_ORIG = 85,
  X_TLV = 88, X_TTY = 89,
  X_Q = 90, X_QD = 102, X_A = 114, X_LA = 126, X_LLA = 138, X_LDV = 150, X_TQ = 162, X_RP = 174,
  // derived
  X_BLV = 186, X_BAV = 189, X_EUL = 192, X_SIN = 195, X_COS = 196, X_ST = 197, X_RESET = 199, X_PF2 = 200,
  X_PT2 = 202, X_CMD2 = 205, X_RV = 209 /* root velocity after the push / reset */, X_PG = 215,
  X_SUM = 218 /* sm1 sm2 sm3 acc vel tq dn jp */, X_RP8 = 226 /* the waves' reward partials */,
  X_NOISE = 234, X_NSLOT = 282
};
// block barrier ordering LDS only (no lane reads a global location another lane of the launch
// wrote), so a phase does not wait for the previous one's global stores to be acknowledged
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
__device__ __forceinline__ float dist_term(float dx, float dy, float lo, float hi) {  // feet / knee distance
  const float d = sqrtf(dx * dx + dy * dy);
  const float dmin = fminf(fmaxf(d - lo, -0.5f), 0.f);
  const float dmax = fminf(fmaxf(d - hi, 0.f), 0.5f);
  return (__expf(-fabsf(dmin) * 100.f) + __expf(-fabsf(dmax) * 100.f)) / 2.f;
}
}  // namespace

__global__ void __launch_bounds__(64 * PWAVES) k_post_step(HgState S, const hg_cfg C, uint64_t counter,
                                                              float* __restrict__ frame_obs, float* __restrict__ frame_priv) {
  __shared__ float xs[X_NSLOT * PEB];
  __shared__ float fo[PEB * HG_OBS1];
  __shared__ float fp[PEB * HG_PRIV1];
  __shared__ float acc_sh[HG_NUM_REWARDS + 1];
  const hg_cfg* cfg = &C;
  const int t = threadIdx.x, l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform job index
  const int np = S.np, n = S.n;
  // XCD-aware: consecutive env groups on one XCD (block b runs on XCD b % 8), so the SoA lines two
  // groups share (PEB < 32: 4 PEB bytes per row) are fetched through one L2
  const int nb = gridDim.x, xcd = blockIdx.x & 7, kx = blockIdx.x >> 3;
  const int e0 = (xcd * (nb >> 3) + min(xcd, nb & 7) + kx) * PEB;
  const bool lane_ok = l < PEB;
  const int e = e0 + (lane_ok ? l : PEB - 1);
  const bool valid = lane_ok && e < n;
  const int ec = min(e, n - 1);  // clamped: loads of the padding lanes stay in bounds
  const int nv = min(PEB, n - e0);
#define X(slot) xs[(slot) * PEB + l]
  const int f0 = C.feet_body[0], f1 = C.feet_body[1];
  const int k0 = C.knee_body[0], k1 = C.knee_body[1];

  // ---------------- L: staging loads
  {
    auto ld = [&](const float* src, int row) { return src[(size_t)row * np + ec]; };
    // observation noise rows [e][48] (64 envs x 12 float4, contiguous), with the counter that says
    // whether the K_step epilogue drew them for this launch
    float4 nz[2];
    bool ready = false;
    if (C.add_noise) {
      const float4* src = reinterpret_cast<const float4*>(S.obs_noise + (size_t)e0 * 48);
#pragma unroll
      for (int i = 0; i < 2; i++) {
        const int q = t + i * 64 * PWAVES;
        nz[i] = q < nv * 12 ? src[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      ready = *S.noise_counter == counter;
    }
    float v[24];
    if (lane_ok) switch (w) {
      case 0:
#pragma unroll
        for (int i = 0; i < 13; i++) v[i] = ld(S.root, i);
#pragma unroll
        for (int i = 0; i < 4; i++) v[13 + i] = ld(S.commands, i);
#pragma unroll
        for (int i = 0; i < 6; i++) v[17 + i] = ld(S.last_root_vel, i);
#pragma unroll
        for (int i = 0; i < 23; i++) X(X_ROOT + i) = v[i];  // root, cmd, lrv are consecutive slots
        break;
      case 1: {
#pragma unroll
        for (int i = 0; i < 2; i++) {
          v[i] = ld(S.feet_air_time, i); v[2 + i] = ld(S.feet_height, i); v[4 + i] = ld(S.last_feet_z, i);
        }
#pragma unroll
        for (int i = 0; i < 3; i++) { v[6 + i] = ld(S.push_force, i); v[9 + i] = ld(S.push_torque, i); v[14 + i] = ld(S.env_origins, i); }
        v[12] = S.friction[ec];
        v[13] = S.body_mass[ec];
        const uint8_t lc0 = S.last_contacts[ec], lc1 = S.last_contacts[np + ec];
        const int ep = reinterpret_cast<const int*>(S.ep_len)[2 * ec];  // low word (0 <= ep_len < 2^31)
        const int tlv = S.terrain_level[ec], tty = S.terrain_type[ec];
#pragma unroll
        for (int i = 0; i < 14; i++) X(X_FAT + i) = v[i];  // fat fht lfz pf pt fric bmass
#pragma unroll
        for (int i = 0; i < 3; i++) X(X_ORIG + i) = v[14 + i];
        X(X_LC) = lc0 ? 1.f : 0.f;
        X(X_LC + 1) = lc1 ? 1.f : 0.f;
        X(X_EP) = __int_as_float(ep + 1);
        X(X_TLV) = __int_as_float(tlv);
        X(X_TTY) = __int_as_float(tty);
        break;
      }
      case 2:
#pragma unroll
        for (int i = 0; i < HG_NUM_REWARDS; i++) v[i] = ld(S.ep_sums, i);
#pragma unroll
        for (int i = 0; i < HG_NUM_REWARDS; i++) X(X_ES + i) = v[i];
        break;
      case 3: case 4: case 5: case 6: {
        const float* a = w == 3 ? S.dof_pos : (w == 4 ? S.actions : (w == 5 ? S.last_last_actions : S.torques));
        const float* b = w == 3 ? S.dof_vel : (w == 4 ? S.last_actions : (w == 5 ? S.last_dof_vel : S.ref_dof_pos));
#pragma unroll
        for (int i = 0; i < 12; i++) { v[i] = ld(a, i); v[12 + i] = ld(b, i); }
        const int base = X_Q + (w - 3) * 24;  // q qd | a la | lla ldv | tq refp
#pragma unroll
        for (int i = 0; i < 24; i++) X(base + i) = v[i];
        break;
      }
      default: {  // contact forces of the base and feet, rigid rows of the feet and knees
#pragma unroll
        for (int i = 0; i < 3; i++) {
          v[i] = ld(S.contact, i);
          v[3 + i] = ld(S.contact, f0 * 3 + i);
          v[6 + i] = ld(S.contact, f1 * 3 + i);
        }
        const int fr[5] = {0, 1, 2, 10, 11};
#pragma unroll
        for (int i = 0; i < 5; i++) { v[9 + i] = ld(S.rigid, f0 * 13 + fr[i]); v[14 + i] = ld(S.rigid, f1 * 13 + fr[i]); }
        v[19] = ld(S.rigid, k0 * 13); v[20] = ld(S.rigid, k0 * 13 + 1);
        v[21] = ld(S.rigid, k1 * 13); v[22] = ld(S.rigid, k1 * 13 + 1);
#pragma unroll
        for (int i = 0; i < 23; i++) X(X_CF + i) = v[i];  // cf then rg are consecutive slots
        break;
      }
    }
    // noise: float4 q of the block is env q / 12, components 4 (q % 12) ..
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int q = t + i * 64 * PWAVES;
      if (q < PEB * 12) {
        const int qe = q / 12, qq = q % 12;
        float* z = &xs[(X_NOISE + 4 * qq) * PEB + qe];
        float zz[4] = {0.f, 0.f, 0.f, 0.f};
        if (C.add_noise) {
          if (ready) {
            zz[0] = nz[i].x; zz[1] = nz[i].y; zz[2] = nz[i].z; zz[3] = nz[i].w;
          } else {
            normals4(rng4(cfg, min(e0 + qe, n - 1), counter, qq, RNG_OBS_NOISE), zz);
          }
        }
        z[0] = zz[0]; z[PEB] = zz[1]; z[2 * PEB] = zz[2]; z[3 * PEB] = zz[3];
      }
    }
    if (t <= HG_NUM_REWARDS) acc_sh[t] = 0.f;
  }
  lds_barrier();

  const int64_t ep = (int64_t)__float_as_int(X(X_EP));
  const float qx = X(X_ROOT + 3), qy = X(X_ROOT + 4), qz = X(X_ROOT + 5), qw = X(X_ROOT + 6);
  // check_termination (:811-816), wherever a wave needs it
  auto reset_flag = [&]() {
    const float c0 = X(X_CF), c1 = X(X_CF + 1), c2 = X(X_CF + 2);
    const float fbn = sqrtf(c0 * c0 + c1 * c1 + c2 * c2);
    return (fbn > 1.0f) || (ep > (int64_t)C.max_episode_length);
  };

  // ---------------- D: derived state, one job per wave
  if (valid) {
    switch (w) {
      case 0: {  // base frame velocities, projected gravity, termination
        const f3 blv = quat_rotate_inverse(qx, qy, qz, qw, mk(X(X_ROOT + 7), X(X_ROOT + 8), X(X_ROOT + 9)));
        const f3 bav = quat_rotate_inverse(qx, qy, qz, qw, mk(X(X_ROOT + 10), X(X_ROOT + 11), X(X_ROOT + 12)));
        const f3 pg = quat_rotate_inverse(qx, qy, qz, qw, mk(0, 0, -1));
        const bool timeout = ep > (int64_t)C.max_episode_length;
        const bool do_reset = reset_flag();
        X(X_BLV) = blv.x; X(X_BLV + 1) = blv.y; X(X_BLV + 2) = blv.z;
        X(X_BAV) = bav.x; X(X_BAV + 1) = bav.y; X(X_BAV + 2) = bav.z;
        X(X_PG) = pg.x; X(X_PG + 1) = pg.y; X(X_PG + 2) = pg.z;
        X(X_RESET) = do_reset ? 1.f : 0.f;
        S.base_lin_vel[e] = blv.x; S.base_lin_vel[np + e] = blv.y; S.base_lin_vel[2 * np + e] = blv.z;
        S.base_ang_vel[e] = bav.x; S.base_ang_vel[np + e] = bav.y; S.base_ang_vel[2 * np + e] = bav.z;
        if (!do_reset) { S.proj_gravity[e] = pg.x; S.proj_gravity[np + e] = pg.y; S.proj_gravity[2 * np + e] = pg.z; }
        S.ep_len[e] = do_reset ? 0 : ep;
        S.time_out[e] = timeout;
        S.reset_buf[e] = do_reset;
        break;
      }
      case 1: {  // euler angles
        const f3 eul = euler_xyz(qx, qy, qz, qw);
        X(X_EUL) = eul.x; X(X_EUL + 1) = eul.y; X(X_EUL + 2) = eul.z;
        break;
      }
      case 2: {  // _resample_commands (:1018-1032), heading command
        float cmd[4] = {X(X_CMD), X(X_CMD + 1), X(X_CMD + 2), X(X_CMD + 3)};
        if ((int)ep % C.resample_interval == 0) {
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
        const bool do_reset = reset_flag();
#pragma unroll
        for (int i = 0; i < 4; i++) { X(X_CMD2 + i) = cmd[i]; if (!do_reset) S.commands[i * np + e] = cmd[i]; }
        break;
      }
      case 3: {  // gait phase
        const Gait g = gait(cfg, ep);
        X(X_SIN) = g.sin_pos; X(X_COS) = g.cos_pos; X(X_ST) = g.stance[0]; X(X_ST + 1) = g.stance[1];
        break;
      }
      case 4: {  // _push_robots (:665-681); the reset lanes rewrite the root
        float pf[2] = {X(X_PF), X(X_PF + 1)}, pt[3] = {X(X_PT), X(X_PT + 1), X(X_PT + 2)};
        float rv[6];
#pragma unroll
        for (int i = 0; i < 6; i++) rv[i] = X(X_ROOT + 7 + i);
        if (C.push_robots && (counter % (uint64_t)C.push_interval == 0)) {
          u4 p0 = rng4(cfg, e, counter, 0, RNG_PUSH), p1 = rng4(cfg, e, counter, 1, RNG_PUSH);
          const float mv = C.max_push_vel_xy, ma = C.max_push_ang_vel;
          pf[0] = 2.f * mv * u01(p0.x) - mv; pf[1] = 2.f * mv * u01(p0.y) - mv;
          rv[0] = pf[0]; rv[1] = pf[1];
          pt[0] = 2.f * ma * u01(p0.z) - ma; pt[1] = 2.f * ma * u01(p0.w) - ma; pt[2] = 2.f * ma * u01(p1.x) - ma;
          rv[3] = pt[0]; rv[4] = pt[1]; rv[5] = pt[2];
          S.push_force[e] = pf[0]; S.push_force[np + e] = pf[1];
          S.push_torque[e] = pt[0]; S.push_torque[np + e] = pt[1]; S.push_torque[2 * np + e] = pt[2];
          if (!reset_flag()) {
            S.root[7 * np + e] = rv[0]; S.root[8 * np + e] = rv[1];
            S.root[10 * np + e] = rv[3]; S.root[11 * np + e] = rv[4]; S.root[12 * np + e] = rv[5];
          }
        }
        X(X_PF2) = pf[0]; X(X_PF2 + 1) = pf[1]; X(X_PT2) = pt[0]; X(X_PT2 + 1) = pt[1]; X(X_PT2 + 2) = pt[2];
#pragma unroll
        for (int i = 0; i < 6; i++) X(X_RV + i) = rv[i];
        break;
      }
      case 5: {  // action smoothness sums
        float t1 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
        for (int j = 0; j < HG_ND; j++) {
          const float a = X(X_A + j), la = X(X_LA + j), lla = X(X_LLA + j);
          float d1 = la - a, d2 = a + lla - 2.f * la;
          t1 += d1 * d1; t2 += d2 * d2; t3 += fabsf(a);
        }
        X(X_SUM) = t1; X(X_SUM + 1) = t2; X(X_SUM + 2) = t3;
        break;
      }
      case 6: {  // dof acc / vel, torques sums
        float sa = 0.f, sv = 0.f, st = 0.f;
#pragma unroll
        for (int j = 0; j < HG_ND; j++) {
          const float qd = X(X_QD + j), tq = X(X_TQ + j);
          float acc = (X(X_LDV + j) - qd) / C.dt;
          sa += acc * acc;
          sv += qd * qd;
          st += tq * tq;
        }
        X(X_SUM + 3) = sa; X(X_SUM + 4) = sv; X(X_SUM + 5) = st;
        break;
      }
      default: {  // default pose, joint position sums
        float dn = 0.f, jp = 0.f;
#pragma unroll
        for (int j = 0; j < HG_ND; j++) {
          const float q = X(X_Q + j);
          float d = q - C.default_dof_pos[j];
          dn += d * d;
          float dj = q - X(X_RP + j);
          jp += dj * dj;
        }
        X(X_SUM + 6) = dn; X(X_SUM + 7) = jp;
        break;
      }
    }
  }
  lds_barrier();

  // ---------------- T: the reward terms (compute_reward :889-907, _reward_* :1170-1437)
  const bool do_reset = X(X_RESET) != 0.f;
  if (valid) {
    float part = 0.f;
    auto add = [&](int k, float term) {  // scaled term into the partial reward and the episode sum
      const float r = term * C.reward_scale[k];
      part += r;
      const float es = X(X_ES + k) + r;
      X(X_ES + k) = es;
      if (!do_reset) S.ep_sums[(size_t)k * np + e] = es;
    };
    const float st0 = X(X_ST), st1 = X(X_ST + 1);
    const float* cfz = &X(X_CF);  // slot stride PEB
    const bool contact[2] = {cfz[5 * PEB] > 5.f, cfz[8 * PEB] > 5.f};
    switch (w) {
      case 0: {  // 0 action_smoothness, 1 base_acc, 2 base_height
        add(0, X(X_SUM) + X(X_SUM + 1) + 0.05f * X(X_SUM + 2));
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < 6; i++) { float d = X(X_LRV + i) - X(X_RV + i); ss += d * d; }
        add(1, __expf(-sqrtf(ss) * 3.f));
        float mh = (X(X_RG + 2) * st0 + X(X_RG + 7) * st1) / (st0 + st1);
        float bh = X(X_ROOT + 2) - (mh - 0.05f);
        add(2, __expf(-fabsf(bh - C.base_height_target) * 100.f));
        break;
      }
      case 1: {  // 3 collision, 4 default_joint_pos, 5 dof_acc, 6 dof_vel, 17 torques
        const float c0 = X(X_CF), c1 = X(X_CF + 1), c2 = X(X_CF + 2);
        add(3, sqrtf(c0 * c0 + c1 * c1 + c2 * c2) > 0.1f ? 1.f : 0.f);
        float dy[4];
#pragma unroll
        for (int m = 0; m < 4; m++) dy[m] = X(X_Q + C.yaw_roll_idx[m]) - C.default_dof_pos[C.yaw_roll_idx[m]];
        float lft = sqrtf(dy[0] * dy[0] + dy[1] * dy[1]);
        float rgt = sqrtf(dy[2] * dy[2] + dy[3] * dy[3]);
        float y = fminf(fmaxf(lft + rgt - 0.1f, 0.f), 50.f);
        add(4, __expf(-y * 100.f) - 0.01f * sqrtf(X(X_SUM + 6)));
        add(5, X(X_SUM + 3));
        add(6, X(X_SUM + 4));
        add(17, X(X_SUM + 5));
        break;
      }
      case 2: {  // 7 feet_air_time (+ last_contacts, feet_air_time)
        float fat[2] = {X(X_FAT), X(X_FAT + 1)};
        bool lc[2] = {X(X_LC) != 0.f, X(X_LC + 1) != 0.f};
        const float st[2] = {st0, st1};
        float r = 0.f;
#pragma unroll
        for (int f = 0; f < 2; f++) {
          bool filt = contact[f] || (st[f] != 0.f) || lc[f];
          float air = fat[f];
          float first = (air > 0.f && filt) ? 1.f : 0.f;
          if (C.reward_scale[7] != 0.f) {
            lc[f] = contact[f];
            air += C.dt;
            r += fminf(fmaxf(air, 0.f), 0.5f) * first;
            fat[f] = filt ? 0.f : air;
          }
        }
        add(7, r);
        S.last_contacts[e] = lc[0]; S.last_contacts[np + e] = lc[1];
        if (!do_reset) { S.feet_air_time[e] = fat[0]; S.feet_air_time[np + e] = fat[1]; }
        break;
      }
      case 3: {  // 8 feet_clearance (+ last_feet_z, feet_height)
        float fht[2] = {X(X_FHT), X(X_FHT + 1)}, lfz[2] = {X(X_LFZ), X(X_LFZ + 1)};
        const float st[2] = {st0, st1};
        const float fzs[2] = {X(X_RG + 2), X(X_RG + 7)};
        float r = 0.f;
#pragma unroll
        for (int f = 0; f < 2; f++) {
          float fz = fzs[f] - 0.05f;
          float fh = fht[f] + (fz - lfz[f]);
          float swing = 1.f - st[f];
          float pos = fabsf(fh - C.target_feet_height) < 0.01f ? 1.f : 0.f;
          r += pos * swing;
          if (C.reward_scale[8] != 0.f) {
            lfz[f] = fz;
            fht[f] = contact[f] ? 0.f : fh;
          }
        }
        add(8, r);
        S.last_feet_z[e] = lfz[0]; S.last_feet_z[np + e] = lfz[1];
        S.feet_height[e] = fht[0]; S.feet_height[np + e] = fht[1];
        break;
      }
      case 4: {  // 9 feet_contact_forces, 10 feet_contact_number, 12 foot_slip
        const float st[2] = {st0, st1};
        float s9 = 0.f, s10 = 0.f, s12 = 0.f;
#pragma unroll
        for (int f = 0; f < 2; f++) {
          const float cx = X(X_CF + 3 + 3 * f), cy = X(X_CF + 4 + 3 * f), cz = X(X_CF + 5 + 3 * f);
          s9 += fminf(fmaxf(sqrtf(cx * cx + cy * cy + cz * cz) - C.max_contact_force, 0.f), 400.f);
          s10 += ((contact[f] ? 1.f : 0.f) == st[f]) ? 1.f : -0.3f;
          const float wx = X(X_RG + 5 * f + 3), wy = X(X_RG + 5 * f + 4);
          s12 += contact[f] ? sqrtf(sqrtf(wx * wx + wy * wy)) : 0.f;
        }
        add(9, s9);
        add(10, s10 / 2.f);
        add(12, s12);
        break;
      }
      case 5:  // 11 feet_distance, 14 knee_distance
        add(11, dist_term(X(X_RG) - X(X_RG + 5), X(X_RG + 1) - X(X_RG + 6), C.min_dist, C.max_dist));
        add(14, dist_term(X(X_RG + 10) - X(X_RG + 12), X(X_RG + 11) - X(X_RG + 13), C.min_dist, C.max_dist / 2.f));
        break;
      case 6: {  // 13 joint_pos, 15 low_speed, 16 orientation
        float nrm = sqrtf(X(X_SUM + 7));
        add(13, __expf(-2.f * nrm) - 0.2f * fminf(fmaxf(nrm, 0.f), 0.5f));
        const float blx = X(X_BLV), cmd0 = X(X_CMD2);
        float as = fabsf(blx), ac = fabsf(cmd0);
        bool low = as < 0.5f * ac, high = as > 1.2f * ac, des = !(low || high);
        bool mis = sgnf(blx) != sgnf(cmd0);
        float q = 0.f;
        if (low) q = -1.f;
        if (high) q = 0.f;
        if (des) q = 1.2f;
        if (mis) q = -2.f;
        add(15, q * (fabsf(cmd0) > 0.1f ? 1.f : 0.f));
        const float pgx = X(X_PG), pgy = X(X_PG + 1);
        add(16, (__expf(-(fabsf(X(X_EUL)) + fabsf(X(X_EUL + 1))) * 10.f) + __expf(-sqrtf(pgx * pgx + pgy * pgy) * 20.f)) / 2.f);
        break;
      }
      default: {  // 18 track_vel_hard, 19 tracking_ang_vel, 20 tracking_lin_vel, 21 vel_mismatch_exp
        const float blx = X(X_BLV), bly = X(X_BLV + 1), blz = X(X_BLV + 2);
        const float bax = X(X_BAV), bay = X(X_BAV + 1), baz = X(X_BAV + 2);
        const float cmd0 = X(X_CMD2), cmd1 = X(X_CMD2 + 1), cmd2 = X(X_CMD2 + 2);
        float ex = cmd0 - blx, ey = cmd1 - bly;
        float lin_err = sqrtf(ex * ex + ey * ey);
        float ang_err = fabsf(cmd2 - baz);
        add(18, (__expf(-lin_err * 10.f) + __expf(-ang_err * 10.f)) / 2.f - 0.2f * (lin_err + ang_err));
        float ae = cmd2 - baz;
        add(19, __expf(-(ae * ae) * C.tracking_sigma));
        add(20, __expf(-(ex * ex + ey * ey) * C.tracking_sigma));
        add(21, (__expf(-(blz * blz) * 10.f) + __expf(-sqrtf(bax * bax + bay * bay) * 5.f)) / 2.f);
        break;
      }
    }
    X(X_RP8 + w) = part;
  }
  lds_barrier();

  // ---------------- R: reset_idx (:1109-1163) for the resetting lanes, one field group per wave
  const bool any_reset = __builtin_amdgcn_ballot_w64(valid && do_reset) != 0;  // wave-uniform
  if (w == 6 && any_reset) {  // episode sums -> this block's statistics: lane k sums term k over the resetting envs
    if (l <= HG_NUM_REWARDS) {
      float tot = 0.f;
      for (int i = 0; i < nv; i++) {
        const bool r = xs[X_RESET * PEB + i] != 0.f;
        tot += r ? (l < HG_NUM_REWARDS ? xs[(X_ES + l) * PEB + i] : 1.f) : 0.f;
      }
      acc_sh[l] = tot;
    }
    if (valid && do_reset) {
#pragma unroll
      for (int k = 0; k < HG_NUM_REWARDS; k++) S.ep_sums[(size_t)k * np + e] = 0.f;
    }
  }
  if (valid) {
    if (w == 7) {  // the reward: the waves' partials in wave order
      float rew = 0.f;
#pragma unroll
      for (int i = 0; i < PWAVES; i++) rew += X(X_RP8 + i);
      if (C.only_positive_rewards) rew = fmaxf(rew, 0.f);
      S.rew[e] = rew;
    }
    if (do_reset) {
      switch (w) {
        case 0: {  // _update_terrain_curriculum (:1075-1095), then _reset_root_states (:1049-1072)
          float org[3] = {X(X_ORIG), X(X_ORIG + 1), X(X_ORIG + 2)};
          if (C.curriculum && counter != 0) {
            const float dx = X(X_ROOT) - org[0], dy = X(X_ROOT + 1) - org[1];
            const float dist = sqrtf(dx * dx + dy * dy);
            const float c0 = X(X_CMD2), c1 = X(X_CMD2 + 1);
            const bool up = dist > C.terrain_env_length / 2;
            const bool down = (dist < sqrtf(c0 * c0 + c1 * c1) * C.max_episode_length_s * 0.5f) && !up;
            int lvl = __float_as_int(X(X_TLV)) + (up ? 1 : 0) - (down ? 1 : 0);
            const int maxl = C.terrain_rows;
            if (lvl >= maxl) {  // torch.randint_like(levels, max_terrain_level)
              lvl = min((int)(u01(rng4(cfg, e, counter, 0, RNG_TERRAIN).x) * (float)maxl), maxl - 1);
            } else {
              lvl = max(lvl, 0);
            }
            S.terrain_level[e] = lvl;
            const float* to = C.terrain_origins + ((size_t)lvl * C.terrain_cols + __float_as_int(X(X_TTY))) * 3;
#pragma unroll
            for (int i = 0; i < 3; i++) { org[i] = to[i]; S.env_origins[i * np + e] = org[i]; }
          }
          float root[13];
#pragma unroll
          for (int i = 0; i < 3; i++) root[i] = C.init_pos[i] + org[i];
#pragma unroll
          for (int i = 0; i < 4; i++) root[3 + i] = C.init_rot[i];
#pragma unroll
          for (int i = 0; i < 3; i++) { root[7 + i] = C.init_lin_vel[i]; root[10 + i] = C.init_ang_vel[i]; }
          if (C.terrain_type != 0) {  // custom origins: xy within 1 m of the centre
            u4 r = rng4(cfg, e, counter, 0, RNG_RESET_ROOT);
            root[0] += 2.0f * u01(r.x) - 1.0f;
            root[1] += 2.0f * u01(r.y) - 1.0f;
          }
          if (C.fix_base_link) {
#pragma unroll
            for (int i = 7; i < 13; i++) root[i] = 0.f;
            root[2] += 1.8f;
          }
#pragma unroll
          for (int i = 0; i < 13; i++) S.root[i * np + e] = root[i];
#pragma unroll
          for (int i = 0; i < 6; i++) X(X_RV + i) = root[7 + i];
          break;
        }
        case 1: case 2: {  // _reset_dofs (:1034-1048): joints 0..5 / 6..11
          auto dofs = [&](const int j0) {
            const u4 ra = rng4(cfg, e, counter, j0 / 4, RNG_RESET_DOF), rb = rng4(cfg, e, counter, j0 / 4 + 1, RNG_RESET_DOF);
            const uint32_t u[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
#pragma unroll
            for (int i = 0; i < 6; i++) {
              const int j = j0 + i;
              const float q = C.default_dof_pos[j] + ((0.1f - (-0.1f)) * u01(u[j - (j0 / 4) * 4]) + (-0.1f));  // default + torch_rand_float(-0.1, 0.1)
              S.dof_pos[j * np + e] = q;
              S.dof_vel[j * np + e] = 0.f;
              S.actions[j * np + e] = 0.f;
              X(X_Q + j) = q; X(X_QD + j) = 0.f; X(X_A + j) = 0.f; X(X_LA + j) = 0.f;
            }
          };
          if (w == 1) dofs(0);
          else dofs(6);
          break;
        }
        case 5: {  // _resample_commands (salt 1); the step's heading command stays in slot 2 or 3
          const u4 r = rng4(cfg, e, counter, 1, RNG_CMD);
          float cmd[4] = {0.f, 0.f, X(X_CMD2 + 2), X(X_CMD2 + 3)};
          const float cx = (C.cmd_lin_x[1] - C.cmd_lin_x[0]) * u01(r.x) + C.cmd_lin_x[0];
          const float cy = (C.cmd_lin_y[1] - C.cmd_lin_y[0]) * u01(r.y) + C.cmd_lin_y[0];
          if (C.heading_command) cmd[3] = (C.cmd_heading[1] - C.cmd_heading[0]) * u01(r.z) + C.cmd_heading[0];
          else cmd[2] = (C.cmd_ang_yaw[1] - C.cmd_ang_yaw[0]) * u01(r.z) + C.cmd_ang_yaw[0];
          const float keep = sqrtf(cx * cx + cy * cy) > 0.2f ? 1.f : 0.f;
          cmd[0] = cx * keep;
          cmd[1] = cy * keep;
#pragma unroll
          for (int i = 0; i < 4; i++) { X(X_CMD2 + i) = cmd[i]; S.commands[i * np + e] = cmd[i]; }
          break;
        }
        case 7: {  // episode counters; the reset root's euler angles, gravity and gait
          S.feet_air_time[e] = 0.f; S.feet_air_time[np + e] = 0.f;
          const f3 eo = euler_xyz(C.init_rot[0], C.init_rot[1], C.init_rot[2], C.init_rot[3]);
          const f3 g = quat_rotate_inverse(C.init_rot[0], C.init_rot[1], C.init_rot[2], C.init_rot[3], mk(0, 0, -1));
          X(X_EUL) = eo.x; X(X_EUL + 1) = eo.y; X(X_EUL + 2) = eo.z;
          S.proj_gravity[e] = g.x; S.proj_gravity[np + e] = g.y; S.proj_gravity[2 * np + e] = g.z;
          const Gait g0 = gait(cfg, 0);
          X(X_SIN) = g0.sin_pos; X(X_COS) = g0.cos_pos; X(X_ST) = g0.stance[0]; X(X_ST + 1) = g0.stance[1];
          break;
        }
        default:
          break;
      }
    }
  }
  if ((w == 3 || w == 4) && any_reset) {  // warm-start impulses: lane -> (env l % PEB, row group l / PEB)
    constexpr int G = 64 / PEB;                // row groups per wave
    const int ei = l % PEB, g = l / PEB;
    const int er = e0 + ei;
    if (er < n && xs[X_RESET * PEB + ei] != 0.f) {
      for (int r = (w - 3) * G + g; r < HG_LAMW; r += 2 * G) S.lambda[(size_t)r * np + er] = 0.f;
    }
  }
  lds_barrier();
  if (t <= HG_NUM_REWARDS && acc_sh[HG_NUM_REWARDS] > 0.f) atomicAdd(&S.ep_stats[24 + t], acc_sh[t]);

  // ---------------- O: observation frames (humanoid_env.py:818-887) in LDS, last_* copies (:802-806)
  const float clip = C.clip_observations;
  auto cl = [clip](float v) { return fminf(fmaxf(v, -clip), clip); };
  if (valid) {
    float* P = fp + l * HG_PRIV1;
    float* O = fo + l * HG_OBS1;
    const float nl = C.noise_level;
    const float sinp = X(X_SIN);
    switch (w) {
      case 0: {  // phase and command slots, base linear velocity, euler angles, last_root_vel
        const float c0 = X(X_CMD2) * C.obs_lin_vel, c1 = X(X_CMD2 + 1) * C.obs_lin_vel, c2 = X(X_CMD2 + 2) * C.obs_ang_vel;
        P[0] = cl(sinp); P[1] = cl(X(X_COS)); P[2] = cl(c0); P[3] = cl(c1); P[4] = cl(c2);
        O[0] = cl(sinp); O[1] = cl(X(X_COS)); O[2] = cl(c0); O[3] = cl(c1); O[4] = cl(c2);
#pragma unroll
        for (int i = 0; i < 3; i++) {
          P[53 + i] = cl(X(X_BLV + i) * C.obs_lin_vel);
          S.base_euler[i * np + e] = X(X_EUL + i);
        }
#pragma unroll
        for (int i = 0; i < 6; i++) S.last_root_vel[i * np + e] = X(X_RV + i);
        break;
      }
      case 1: case 2: case 3: {  // joints 4 (w - 1) .. +3: compute_ref_state (:705-744), frames, last_*
        const float sl = fminf(sinp, 0.f), sr = fmaxf(sinp, 0.f);
        const float s1 = C.target_joint_pos_scale, s2 = 2.f * s1;
        const bool zero = fabsf(sinp) < 0.1f;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int j = (w - 1) * 4 + i;
          // the later assignment wins when indices coincide, as the reference's sequential stores
          float v = 0.f;
          v = (j == C.ref_idx[0]) ? sl * s1 : v;
          v = (j == C.ref_idx[1]) ? sl * s2 : v;
          v = (j == C.ref_idx[2]) ? sl * s1 : v;
          v = (j == C.ref_idx[3]) ? sr * s1 : v;
          v = (j == C.ref_idx[4]) ? sr * s2 : v;
          v = (j == C.ref_idx[5]) ? sr * s1 : v;
          const float ref = zero ? 0.f : v;
          S.ref_dof_pos[j * np + e] = ref;
          const float q = X(X_Q + j), qd = X(X_QD + j), a = X(X_A + j);
          const float dq = q - C.default_dof_pos[j];
          P[5 + j] = cl(dq * C.obs_dof_pos);
          P[17 + j] = cl(qd * C.obs_dof_vel);
          P[29 + j] = cl(a);
          P[41 + j] = cl(q - ref);
          O[5 + j] = cl(dq * C.obs_dof_pos + X(X_NOISE + 5 + j) * (C.noise_dof_pos * C.obs_dof_pos) * nl);
          O[17 + j] = cl(qd * C.obs_dof_vel + X(X_NOISE + 17 + j) * (C.noise_dof_vel * C.obs_dof_vel) * nl);
          O[29 + j] = cl(a);
          S.last_last_actions[j * np + e] = X(X_LA + j);
          S.last_actions[j * np + e] = a;
          S.last_dof_vel[j * np + e] = qd;
        }
        break;
      }
      case 4: {  // angular velocity, euler angles
#pragma unroll
        for (int i = 0; i < 3; i++) {
          P[56 + i] = cl(X(X_BAV + i) * C.obs_ang_vel);
          P[59 + i] = cl(X(X_EUL + i) * C.obs_quat);
          O[41 + i] = cl(X(X_BAV + i) * C.obs_ang_vel + X(X_NOISE + 41 + i) * (C.noise_ang_vel * C.obs_ang_vel) * nl);
          O[44 + i] = cl(X(X_EUL + i) * C.obs_quat + X(X_NOISE + 44 + i) * (C.noise_quat * C.obs_quat) * nl);
        }
        break;
      }
      case 5: {  // push, friction, mass, stance, contact mask
        P[62] = cl(X(X_PF2)); P[63] = cl(X(X_PF2 + 1));
        P[64] = cl(X(X_PT2)); P[65] = cl(X(X_PT2 + 1)); P[66] = cl(X(X_PT2 + 2));
        P[67] = cl(X(X_FRIC));
        P[68] = cl(X(X_BMASS) / 30.f);
        P[69] = X(X_ST); P[70] = X(X_ST + 1);
        P[71] = X(X_CF + 5) > 5.f ? 1.f : 0.f; P[72] = X(X_CF + 8) > 5.f ? 1.f : 0.f;
        break;
      }
      default:
        break;
    }
  }
  lds_barrier();
  // the frames, row-major [e][47] / [e][73]: contiguous over the block's envs
  {
    float* go = frame_obs + (size_t)e0 * HG_OBS1;
    float* gp = frame_priv + (size_t)e0 * HG_PRIV1;
    if (nv == PEB) {  // 16-byte aligned (arena offsets are 256-aligned; 16 * 47 * 4 and 16 * 73 * 4 are multiples of 16)
      for (int q = t; q < PEB * HG_OBS1 / 4; q += 64 * PWAVES)
        reinterpret_cast<float4*>(go)[q] = reinterpret_cast<const float4*>(fo)[q];
      for (int q = t; q < PEB * HG_PRIV1 / 4; q += 64 * PWAVES)
        reinterpret_cast<float4*>(gp)[q] = reinterpret_cast<const float4*>(fp)[q];
    } else {
      for (int q = t; q < nv * HG_OBS1; q += 64 * PWAVES) go[q] = fo[q];
      for (int q = t; q < nv * HG_PRIV1; q += 64 * PWAVES) gp[q] = fp[q];
    }
  }
#undef X
}

// history windows (HgWindow, hg_api.hip): the reference's deque append + stack
// (humanoid_env.py:880-887, history zeroed on reset) as one frame write per (env, table) into the
// row's sliding window instead of a copy of the whole stack; one block per (env, table) row.  The
// last block also folds the episode statistics (ep_stats[k] = acc[k] / n_reset / episode_length_s
// when any env reset) and clears the accumulators.
constexpr int WIN_ROWS = 4;  // (env, table) rows per k_window_stats block, one wave each
__global__ void __launch_bounds__(64 * WIN_ROWS) k_window_stats(HgWindow A, HgWindow B, const float* __restrict__ frame_a,
                                                      const float* __restrict__ frame_b,
                                                      const uint8_t* __restrict__ reset, int n, float* ep_stats,
                                                      float inv_len_s, int ring_slot,
                                                      const int32_t* __restrict__ env_rows,
                                                      int32_t* __restrict__ env_order, int nsort, HgSink sink,
                                                      const float* __restrict__ rew,
                                                      const uint8_t* __restrict__ time_out, int nsink) {
  static_assert(64 * WIN_ROWS == HG_ORD_T, "the order blocks use the window block's threads");
  // blocks 0 .. nsort - 1: the next K_step's env order (hg_common.h), first so that they start
  // with the launch and run beside the window rows
  if ((int)blockIdx.x < nsort) {
    hg_env_order_block(env_rows, env_order, n, blockIdx.x);
    return;
  }
  // blocks nsort .. nsort + nsink - 1: the step's rewards / dones / time-outs into the rollout
  // storage slot (hg_set_rollout_sink; hg_rollout_env's writes with the bootstrap deferred)
  if ((int)blockIdx.x < nsort + nsink) {
    const int e = ((int)blockIdx.x - nsort) * (64 * WIN_ROWS) + (int)threadIdx.x;
    if (e < n) {
      sink.rew[e] = rew[e];
      sink.dones[e] = reset[e];
      if (sink.time_outs) sink.time_outs[e] = time_out[e];
    }
    return;
  }
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
  // one wave per (env, table) row, WIN_ROWS rows per block
  const int b = (blockIdx.x - nsort - nsink) * WIN_ROWS + (threadIdx.x >> 6);
  if (b >= 2 * n) return;
  const int lane = threadIdx.x & 63;
  const bool a = b < n;
  const HgWindow& T = a ? A : B;
  const int e = a ? b : b - n;
  const float* __restrict__ fr = (a ? frame_a : frame_b) + (size_t)e * T.width;
  float* __restrict__ row = T.win + (size_t)e * T.rowlen;
  const int hist = (T.frames - 1) * T.width;  // the older frames of the new stack
  const bool rs = reset[e] != 0;
  float* __restrict__ h0 = row + (size_t)T.head * T.width;
  if (T.shift_src >= 0) {  // h0 == row; source and destination slots do not overlap (HW >= frames - 1)
    const float* __restrict__ src = row + (size_t)T.shift_src * T.width;
    for (int k = lane; k < hist; k += 64) h0[k] = rs ? 0.f : src[k];
  } else if (rs) {
    for (int k = lane; k < hist; k += 64) h0[k] = 0.f;
  }
  for (int k = lane; k < T.width; k += 64) h0[hist + k] = fr[k];
}

extern "C" int hg_launch_post(const HgState* S, const hg_cfg* hcfg, uint64_t counter, int mode, const uint8_t* mask,
                              float* frame_obs, float* frame_priv, HgWindow obs, HgWindow priv, float inv_len_s,
                              int ep_slot, HgSink sink, hipStream_t stream) {
  const int n = S->n;
  if (mode == 0)
    hipLaunchKernelGGL(k_post_step, dim3((n + PEB - 1) / PEB), dim3(64 * PWAVES), 0, stream, *S, *hcfg, counter,
                       frame_obs, frame_priv);
  else
    hipLaunchKernelGGL(k_post, dim3((n + 63) / 64), dim3(64), 0, stream, *S, counter, mode, mask, frame_obs,
                       frame_priv);
  // the env-order blocks (K_step's wave balancing), WIN_ROWS (env, table) rows per block, the
  // statistics block
  const int nsort = S->balance ? 8 : 0;
  const int nsink = sink.rew ? (n + 64 * WIN_ROWS - 1) / (64 * WIN_ROWS) : 0;
  const int g = nsort + nsink + (2 * n + WIN_ROWS - 1) / WIN_ROWS + 1;
  hipLaunchKernelGGL(k_window_stats, dim3(g), dim3(64 * WIN_ROWS), 0, stream, obs, priv, frame_obs, frame_priv,
                     S->reset_buf, n, S->ep_stats, inv_len_s, ep_slot, S->env_rows, S->env_order, nsort, sink, S->rew,
                     S->time_out, nsink);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
