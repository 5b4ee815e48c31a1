"""Floating-base divergence envelope (GPU vs f64, CPU f32 vs f64) at selected steps (dev tool)."""
import sys
import numpy as np
sys.path.insert(0, "scripts")
import trajectory_curve as TC  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
o = TC.run(False, steps)
g = np.maximum.accumulate(np.array(o["gpu_vs_f64_q"]))
f = np.maximum.accumulate(np.array(o["f32_ensemble_vs_f64_q"]))
for t in list(range(0, 60, 4)) + list(range(60, steps, 10)):
    print(t, f"gpu {g[t]:.2e} f32 {f[t]:.2e} ratio {(g[t] - 1e-5) / f[t]:.2f}")
