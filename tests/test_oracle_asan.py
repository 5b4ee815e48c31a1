"""Sanitizer run of the CPU reference physics (ASan/UBSan on host code).

`make -C oracle asan` builds physics_ref.c (f64 and f32) with AddressSanitizer and
UndefinedBehaviorSanitizer into a standalone driver (oracle/asan_driver.c).  Each scenario below
is written to a file, stepped by that executable (any sanitizer report aborts it with a non-zero
status) and its outputs are compared with the production oracle library libphysref.so on the
same inputs.  Scenarios cover what the physics tests exercise: the production profile on the
plane (all 13 self-collision pairs, joint friction, random poses that touch the ground, the legs
and the hands), a falling base that reaches the base-box corners, and the heightfield."""
import os
import struct
import subprocess

import numpy as np
import pytest

import physics_ref as P
from humanoid import _native as N

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE = os.path.join(os.path.dirname(HERE), "oracle")
EXE = os.path.join(ORACLE, "_asan", "physref_asan")


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", ORACLE, "asan"], check=True)
    return EXE


def _cfg_model(n, heightfield=None):
    from humanoid.envs import XBotLCfg
    from humanoid.envs.custom.humanoid_env import build_hg_cfg
    cfg = XBotLCfg()
    model, js = N.load_model(armature=cfg.sim.hg.armature)
    hf_shape = (0, 0) if heightfield is None else heightfield.shape
    hc, _ = build_hg_cfg(cfg, n, cfg.sim.dt, 5, js, heightfield=None if heightfield is None else 1,
                         hf_shape=hf_shape)
    hc.heightfield = None
    return hc, model


def _scenario(n, steps, seed, fall=False, heightfield=None):
    rng = np.random.default_rng(seed)
    hc, model = _cfg_model(n, heightfield)
    root = np.zeros((n, 13))
    root[:, 2] = 0.95 if not fall else rng.uniform(0.3, 0.6, n)
    ax = rng.standard_normal((n, 3))
    ang = rng.uniform(0, 0.6 if fall else 0.15, n)
    ax /= np.linalg.norm(ax, axis=1, keepdims=True)
    root[:, 3:6] = ax * np.sin(ang / 2)[:, None]
    root[:, 6] = np.cos(ang / 2)
    root[:, 7:13] = rng.standard_normal((n, 6)) * 0.3
    if heightfield is not None:
        root[:, 0:2] = rng.uniform(-20.0, -5.0, (n, 2))  # x + border (25 m) inside the 24 m map
        root[:, 2] += heightfield.max() * hc.hf_vertical_scale
    lo = np.array([model.lower[b + 1] for b in range(12)])
    hi = np.array([model.upper[b + 1] for b in range(12)])
    q = lo + (hi - lo) * rng.uniform(0.1, 0.9, (n, 12))
    qd = rng.standard_normal((n, 12))
    mass0 = model.mass[0] + rng.uniform(-5, 5, n)
    fric = rng.uniform(0.1, 2.0, n)
    act = rng.standard_normal((steps, n, 12)) * 0.5
    return hc, model, root, q, qd, mass0, fric, act


def _run_asan(exe, tmp_path, hc, model, hf, root, q, qd, mass0, fric, act):
    n, steps = root.shape[0], act.shape[0]
    hr, hcol = (0, 0) if hf is None else hf.shape
    src, dst = tmp_path / "scenario.bin", tmp_path / "out.bin"
    with open(src, "wb") as f:
        f.write(struct.pack("<4i", n, steps, hr, hcol))
        f.write(bytes(hc))
        f.write(bytes(model))
        if hf is not None:
            f.write(np.ascontiguousarray(hf, np.int16).tobytes())
        for a in (root, q, qd, mass0, fric, act):
            f.write(np.ascontiguousarray(a, np.float64).tobytes())
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, str(src), str(dst)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, \
        r.stderr[-4000:]
    raw = open(dst, "rb").read()
    out, off = {}, 0
    for prec in ("f64", "f32"):
        for name, cnt in (("root", n * 13), ("q", n * 12), ("qd", n * 12), ("torques", n * 12),
                          ("contact", n * 39)):
            out[prec, name] = np.frombuffer(raw, np.float64, cnt, off)
            off += 8 * cnt
        for name in ("nonfinite", "dropped"):
            out[prec, name] = np.frombuffer(raw, np.int32, n, off)
            off += 4 * n
    assert off == len(raw)
    return out


def _run_lib(hc, model, hf, root, q, qd, mass0, fric, act, prec):
    n = root.shape[0]
    sim = P.RefSim(hc, model, n, prec, heightfield=hf)
    sim.root[:], sim.q[:], sim.qd[:] = root, q, qd
    sim.mass0[:], sim.fric[:] = mass0, fric
    for a in act:
        sim.step(a)
    return {"root": sim.root, "q": sim.q, "qd": sim.qd, "torques": sim.torques, "contact": sim.contact,
            "nonfinite": sim.nonfinite, "dropped": sim.dropped}


def _heightfield():
    rng = np.random.default_rng(7)
    hf = np.cumsum(rng.integers(-3, 4, (240, 240)), axis=0).astype(np.int16)
    return hf - hf.min()


@pytest.mark.parametrize("case", ["plane", "falling", "heightfield"])
def test_physics_oracle_clean_under_asan_ubsan(exe, tmp_path, case):
    hf = _heightfield() if case == "heightfield" else None
    n, steps = (24, 30) if case != "heightfield" else (12, 20)
    args = _scenario(n, steps, seed={"plane": 1, "falling": 2, "heightfield": 3}[case], fall=case == "falling",
                     heightfield=hf)
    hc, model = args[0], args[1]
    san = _run_asan(exe, tmp_path, hc, model, hf, *args[2:])
    for prec in ("f64", "f32"):
        ref = _run_lib(hc, model, hf, *args[2:], prec)
        for name, v in ref.items():
            x = san[prec, name].reshape(v.shape)
            # same source and operation order; only -O1 vs -O2 code generation differs
            np.testing.assert_allclose(x, v.astype(np.float64), rtol=1e-9 if prec == "f64" else 1e-5,
                                       atol=1e-9 if prec == "f64" else 1e-5, err_msg=f"{case} {prec} {name}")
        assert not ref["nonfinite"].any()
    # the scenarios reach the contact and collision code
    assert np.abs(san["f64", "contact"]).sum() > 0
