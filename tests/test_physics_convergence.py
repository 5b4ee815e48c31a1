"""Time-step convergence of the build's physics (quantifies the modelling choice of DESIGN §4):
the Isaac Gym asset runs at armature 0 (humanoid_config.py:118) with kd = 10 on a 0.0015 kg m^2
foot, which explicit integration cannot hold at dt = 1 ms, so the build integrates the PD damping
implicitly (M + dt kd on the diagonal).  These CPU checks run the f64 oracle (the same algorithm as
K_step) on the production gains and limits at dt = 1, 1/2, 1/4, 1/8 and 1/16 ms with the policy
step fixed at 10 ms; as dt shrinks the implicit term vanishes and the trajectories converge, so
the distance of the 1 ms trajectory from the 1/16 ms one is the integrator error of the production
step.  Also measured: how far the MJCF's armature 0.01 (XBot-L.xml:37-39) moves the trajectory.

Fixed base (variant A of SURVEY 8(d): no contact chaos) for 1 s of the open-loop sinusoid.
``HG_CONVERGENCE_OUT=<file>`` writes the numbers as JSON (profiles/r2_v2/physics_convergence.json)."""
import json
import os

import numpy as np
import pytest

import physics_ref as P
from humanoid import _native as N

STEPS = 100
DTS = (1e-3, 5e-4, 2.5e-4, 1.25e-4, 6.25e-5)


def _cfg(n, dt, fixed=True):
    from humanoid.envs import XBotLCfg
    from humanoid.envs.custom.humanoid_env import build_hg_cfg
    cfg = XBotLCfg()
    cfg.asset.fix_base_link = fixed
    cfg.domain_rand.dynamic_randomization = 0.0
    _, js = N.load_model()
    c, _ = build_hg_cfg(cfg, n, dt, 5, js)
    c.decimation = int(round(0.01 / dt))
    c.sim_dt = dt
    return c


def _traj(dt, armature=0.0, fixed=True, steps=STEPS, n=2):
    m, _ = N.load_model(armature=armature)
    c = _cfg(n, dt, fixed)
    sim = P.RefSim(c, m, n, "f64")
    sim.root[:, 2] = 0.95 if not fixed else 1.2
    j = np.arange(12)
    qs, taus = [], []
    for t in range(steps):
        a = np.tile(0.5 * np.sin(2 * np.pi * t * 0.01 / 0.64 + j * np.pi / 6), (n, 1))
        sim.step(a)
        assert not sim.nonfinite.any()
        qs.append(sim.q[0].copy())
        taus.append(sim.torques[0].copy())
    return np.array(qs), np.array(taus)


@pytest.fixture(scope="module")
def trajectories():
    return {dt: _traj(dt) for dt in DTS}


def test_step_convergence(trajectories):
    ref_q, ref_tau = trajectories[DTS[-1]]
    err = {dt: float(np.abs(trajectories[dt][0] - ref_q).max()) for dt in DTS[:-1]}
    errt = {dt: float(np.abs(trajectories[dt][1] - ref_tau).max()) for dt in DTS[:-1]}
    # the error shrinks as dt does (first order: about halves per halving, allowing for the
    # reference's own error at 1/16 ms)
    e = [err[dt] for dt in DTS[:-1]]
    assert all(e[i + 1] < e[i] for i in range(len(e) - 1)), err
    assert e[0] / e[2] > 2.5, err
    # the production step (1 ms) stays within 2e-3 rad of the converged trajectory over 1 s
    # (measured 7.9e-4 rad, 2.3 N m)
    assert e[0] < 2e-3, err
    arm_q, _ = _traj(1e-3, armature=0.01)
    d_arm = float(np.abs(arm_q - trajectories[1e-3][0]).max())
    out = os.environ.get("HG_CONVERGENCE_OUT")
    if out:
        with open(out, "w") as f:
            json.dump({"what": "fixed-base 1 s open-loop sinusoid, production gains/limits, f64 oracle; max |q - q(dt=1/16 ms)| "
                               "and |tau - tau(dt=1/16 ms)| over the trajectory",
                       "max_abs_dq_rad": {f"{dt * 1e3:g} ms": v for dt, v in err.items()},
                       "max_abs_dtau_Nm": {f"{dt * 1e3:g} ms": v for dt, v in errt.items()},
                       "armature_0.01_vs_0_at_1ms_max_abs_dq_rad": d_arm}, f, indent=1)
