#!/bin/bash
# End-to-end training run on one MI355X (4096 envs, the task's defaults: T = 60, 2 epochs x 4
# minibatches) followed by the evaluation scripts on the trained policy: play.py (export +
# headless play) and sim2sim.py on the training (URDF) and the MJCF parameter profiles.
# Everything judged is copied under gpurun_out/train_eval/.  Stops at the first failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R/humanoid-gym-with-comments_amd" || exit 1
OUT="$R/gpurun_out/train_eval"
mkdir -p "$OUT"
ITERS=${ITERS:-1500}
timeout -k 10 ${TRAIN_TIMEOUT:-700} python -m humanoid.scripts.train --task humanoid_ppo --headless --run_name te \
  --max_iterations $ITERS > "$OUT/train.log" 2>&1 || { tail -30 "$OUT/train.log"; exit 1; }
RUN=$(ls -td logs/XBot_ppo/*te | head -n 1)
cp "$RUN/scalars.jsonl" "$OUT/" 2>/dev/null
timeout -k 10 300 python -m humanoid.scripts.play --task humanoid_ppo --headless --resume --steps 300 > "$OUT/play.log" 2>&1 || { tail -30 "$OUT/play.log"; exit 1; }
POL=logs/XBot_ppo/exported/policies/policy_1.pt
cp "$POL" "$OUT/" && cp logs/XBot_ppo/exported/policies/policy.onnx "$OUT/"
for P in urdf mjcf; do
  timeout -k 10 300 python -m humanoid.scripts.sim2sim --load_model "$POL" --profile $P --duration 20 \
    --vx -0.25 0.0 0.3 0.5 --envs_per_command 64 --out "$OUT/sim2sim_$P" > "$OUT/sim2sim_$P.log" 2>&1 \
    || { tail -30 "$OUT/sim2sim_$P.log"; exit 1; }
  tail -6 "$OUT/sim2sim_$P.log"
done
grep -E "Mean reward|Mean episode length|Learning iteration" "$OUT/train.log" | tail -3
