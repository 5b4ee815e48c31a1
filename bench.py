"""Headline benchmark: env-steps/s (whole node) of the full PPO loop at 4096 envs per GPU.

A "step" here is one PPO iteration of the reference's OnPolicyRunner.learn
(humanoid/algo/ppo/on_policy_runner.py:110-170): T=24 x [policy act -> env.step (K_step: 10
physics substeps + K_post: rewards/obs/reset) -> process_env_step], then GAE (K_gae) and the PPO
update (2 epochs x 4 minibatches).  value = envs_per_gpu * T * n_gpus * K / max-over-ranks time,
i.e. the reference's Perf/total_fps summed over the node.  Workload: BASELINE.json configs[1]
(XBot-L, flat terrain, 4096 envs/GPU, 24-step rollout), synthetic data (random-init policy,
no checkpoint), all physics/env inputs resident in HBM.

Multi-GPU: one process per GPU (torch.distributed.run), envs sharded (4096 per rank, weak
scaling), policy gradients all-reduced with RCCL (backend "nccl") once per minibatch.

The roofline object is for the dominant kernel, K_step (FP32 bound, VALU + f32 MFMA: state lives
in registers/LDS across the 10 substeps, algorithmic HBM traffic ~1.8 KB/env-step); its launch
time is measured with HIP events recorded on the stream the kernel runs on (torch's current
stream, which the env passes to hg_step).  ``traffic`` is the HBM bytes per K_step launch from
the committed rocprofv3 PMC passes (profiles/<round>/pmc_summary.json: FETCH_SIZE doubled per
MI355X_MICROARCH.md + WRITE_SIZE), for the same workload.  cpu_baseline times the oracle port (C reference physics,
numpy env logic, torch-CPU PPO) on a bounded sample on the host cores.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector (= FP32 matrix) dense peak
HBM_PEAK_GBS = 8000.0
# K_step algorithmic HBM bytes per env and launch: 828 B read (policy actions,
# previous actions, dof pos / vel, root, 144 warm-start impulses, mass, friction) + 1844 B written
# (actions, rigid 13x13, contacts 13x3, root, dof pos / vel, torques, 144 warm-start impulses, and
# the next post launch's 48 observation-noise normals)
KSTEP_BYTES_PER_ENV = 828 + 1844
PROFILE_DIR = "r6_v3"  # the committed rocprofv3 summaries of the current kernels
PMC_SUMMARY = os.path.join(REPO, "profiles", PROFILE_DIR, "pmc_summary.json")


def sq_issue(kernel_file=os.path.join(REPO, "profiles", PROFILE_DIR, "sq_counters_k_step.json")):
    """SIMD VALU issue utilisation of K_step from the committed SQ counter passes (None if absent)."""
    try:
        with open(kernel_file) as f:
            return json.load(f)["simd_valu_busy_est"]
    except (OSError, KeyError, ValueError):
        return None


def mfma_stats(rows, envs, decimation=10, nf=18,
               kernel_file=os.path.join(REPO, "profiles", PROFILE_DIR, "sq_counters_k_step.json")):
    """K_step's matrix-core use (the Delassus block W = Z^T Z, v_mfma_f32_32x32x2_f32: 32 x 32 x 2
    per instruction = 4096 FLOP, 16 quad-cycles of the SIMD's MFMA pipe) from the committed SQ
    counters: instructions per wave, issued vs useful FLOP (useful = rows^2 nf multiply-adds per env
    and substep at the measured active rows; the 32 x 32 tile covers 32 rows) and the pipe busy
    estimate 2 waves/SIMD x SQ_INSTS_MFMA x 16 / SQ_WAVE_CYCLES (quad-cycles)."""
    try:
        with open(kernel_file) as f:
            pw = json.load(f)["per_wave"]
        n_mfma, wave_cycles = float(pw["SQ_INSTS_MFMA"]), float(pw["SQ_WAVE_CYCLES"])
    except (OSError, KeyError, ValueError):
        return None
    waves = (envs + 1) // 2
    issued = n_mfma * 4096.0 * waves
    useful = 2.0 * rows * rows * nf * decimation * envs
    return {"instr": "v_mfma_f32_32x32x2_f32", "instructions_per_wave": n_mfma,
            "issued_flop_per_launch": issued, "useful_flop_per_launch": round(useful, 1),
            "tile_util": round(useful / issued, 4) if issued else None,
            "pipe_busy_est": round(2.0 * n_mfma * 16.0 / wave_cycles, 4),
            "source": os.path.relpath(kernel_file, REPO)}


def pmc_traffic(kernel="k_step"):
    """HBM bytes per launch of `kernel` from the committed PMC summary (None if absent)."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)[kernel]
        return int(d["hbm_bytes_per_launch_corrected"]), os.path.relpath(PMC_SUMMARY, REPO)
    except (OSError, KeyError, ValueError):
        return None, None


class KernelTimer:
    """HIP-event pairs around kernel launches on the current stream, on one launch in `every`
    (each event record is a barrier packet on the queue: timing every launch would add ~15 us of
    queue gaps per env step to the measured loop)."""

    def __init__(self, every=4):
        self.events = {}
        self.enabled = False
        self.every = every
        self._calls = {}
        self._open = {}

    def start(self, name):
        if not self.enabled:
            return
        k = self._calls.get(name, 0)
        self._calls[name] = k + 1
        self._open[name] = k % self.every == 0
        if not self._open[name]:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.events.setdefault(name, []).append([e, None])

    def stop(self, name):
        if not self.enabled or not self._open.get(name):
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.events[name][-1][1] = e

    def mean_ms(self, name):
        pairs = self.events.get(name, [])
        return float(np.mean([a.elapsed_time(b) for a, b in pairs])) if pairs else float("nan")

    def count(self, name):
        return len(self.events.get(name, []))


def physics_flops_per_env_step(rows, decimation=10, sweeps=5, nf=18):
    """Analytic FLOP count of the K_step algorithm, per env and policy step.
    Per substep: kinematics 3.3k + bias forces (RNEA) 1.8k + joint-space inertia (CRBA) 1.5k +
    Cholesky of the nf x nf legs-first arrow matrix 2.0k + g = L^-1 (tau - h) and the back
    substitution 0.65k + integration 0.1k; per constraint row: the Jacobian row 0.12k, its forward
    solve z = L^-1 J^T (nf^2 = 324 FMA -> 0.65k), the Delassus row W = Z^T Z on MFMA (2 nf rows),
    diagonal / bounds / warm start 0.07k; per PGS sweep and row: the W row times the impulses
    (2 rows) + the update and clamp (12).  Plus one end-of-step FK + quaternions (4.0k)."""
    per_sub = 9350 + rows * (120 + 2 * nf * nf + 2 * nf * rows + 72) + sweeps * rows * (2 * rows + 12)
    return decimation * per_sub + 4000


def active_rows(env):
    """Mean constraint rows per env of the last solve, from the warm-start impulse table
    (HG_LAMW layout, csrc/hg_physics.hip: [0, 72) ground contacts x 3, [72, 120) self-collision
    pair contacts x 3, [120, 132) joint limits, [132, 144) joint-friction rows): a contact with a
    positive normal impulse holds 3 rows, an active limit 1, every joint with friction 1 (always
    solved)."""
    from humanoid import _native as N
    lam = env._view(N.T["CONTACT_LAMBDA"])
    nc3 = (N.HG_MAX_CONTACTS + N.HG_MAX_PAIRS) * 3
    contacts = (lam[:, 0:nc3:3] > 0).sum(dim=1).float()
    limits = (lam[:, nc3:nc3 + N.HG_MAX_DOF] != 0).sum(dim=1).float()
    fric = sum(1 for b in range(len(env._model.joint_friction)) if env._model.joint_friction[b] > 0)
    return float((3 * contacts + limits).mean().item() + fric)


def make_env(num_envs, device, seed, terrain="plane", push_curriculum=False, env_offset=0, num_envs_total=None):
    from humanoid.envs import XBotLCfg
    from humanoid.envs.custom.humanoid_env import XBotLFreeEnv
    from humanoid.utils.helpers import SimParams
    cfg = XBotLCfg()
    cfg.env.num_envs = num_envs
    cfg.seed = seed
    cfg.terrain.mesh_type = terrain
    cfg.terrain.seed = 5  # identical heightfield on every rank
    cfg.domain_rand.push_curriculum = push_curriculum
    cfg.env.env_offset = env_offset          # this rank's shard of the global envs
    cfg.env.num_envs_total = num_envs_total
    return XBotLFreeEnv(cfg, SimParams(), "hg_sim", device, True)


def train_cfg(T, policy_dtype="fp32", obs_dtype="fp32"):
    from humanoid.envs import XBotLCfgPPO
    from humanoid.utils.helpers import class_to_dict
    t = XBotLCfgPPO()
    t.runner.num_steps_per_env = T
    t.policy.policy_dtype = policy_dtype
    t.runner.storage_obs_dtype = obs_dtype
    return class_to_dict(t)


def host_cores():
    """Host threads the baseline may use: OMP_NUM_THREADS when set (the GPU box's CPU share, 16),
    else the CPUs this process may run on."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(n_envs=256, T=24, threads=None, iterations=3):
    """The oracle port on the host: C reference physics (f32, OpenMP over envs), numpy env logic
    (oracle/pipeline_ref.py), torch-CPU policy + GAE + PPO update — `iterations` full PPO
    iterations on n_envs envs after the set-up.  Returns (env-steps/s, threads, seconds)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import physics_ref as P
    import pipeline_ref as PR
    import envlogic_ref as E
    from humanoid import _native as N
    from humanoid.envs import XBotLCfg
    from humanoid.envs.custom.humanoid_env import build_hg_cfg
    from humanoid.algo.ppo import ActorCritic, PPO
    threads = threads or host_cores()
    torch.set_num_threads(threads)
    os.environ["OMP_NUM_THREADS"] = str(threads)
    P.set_threads(threads)
    cfg = XBotLCfg()
    model, js = N.load_model(armature=cfg.sim.hg.armature)
    hc, _ = build_hg_cfg(cfg, n_envs, cfg.sim.dt, 5, js)
    oc = PR.Cfg(hc)
    side = int(np.ceil(np.sqrt(n_envs)))
    origins = np.zeros((n_envs, 3), np.float32)
    origins[:, 0] = 3.0 * (np.arange(n_envs) // side)
    origins[:, 1] = 3.0 * (np.arange(n_envs) % side)
    rng = np.random.default_rng(5)
    mass = model.mass[0] + rng.uniform(-5, 5, n_envs)
    fric = rng.uniform(0.1, 2.0, n_envs)
    S, obs, priv = PR.initial_state(oc, origins, mass, fric)
    sim = P.RefSim(hc, model, n_envs, "f32")
    sim.mass0[:] = mass
    sim.fric[:] = fric
    torch.manual_seed(5)
    ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128])
    ppo = PPO(ac, num_learning_epochs=2, num_mini_batches=4, clip_param=0.2, gamma=0.994, lam=0.9,
              learning_rate=1e-5, entropy_coef=0.001, schedule="adaptive", desired_kl=0.01, device="cpu")
    ppo.init_storage(n_envs, T, [705], [219], [12])
    ppo.storage.gae_fn = lambda r, d, v, lv, g, l: tuple(
        torch.from_numpy(x)[..., None] for x in E.gae(r[..., 0].numpy(), d[..., 0].numpy(), v[..., 0].numpy(),
                                                      lv[:, 0].numpy(), g, l, normalize=False))
    t0 = time.time()
    counter = 0
    for _ in range(iterations):
        with torch.inference_mode():
            for _ in range(T):
                a = ppo.act(torch.from_numpy(obs), torch.from_numpy(priv)).numpy()
                a_ref = PR.preprocess_actions(oc, a, S["actions"], counter)
                S["actions"] = a_ref
                sim.root[:], sim.q[:], sim.qd[:], sim.lam[:] = S["root_states"], S["dof_pos"], S["dof_vel"], S["lambda"]
                sim.step(a_ref)
                S.update(root_states=sim.root.copy(), dof_pos=sim.q.copy(), dof_vel=sim.qd.copy(),
                         torques=sim.torques.copy(), contact_forces=sim.contact.copy(), rigid_state=sim.rigid.copy())
                S["lambda"] = sim.lam.copy()
                counter += 1
                obs, priv, rew, reset, timeout, _ = PR.post(oc, S, counter, obs, priv)
                infos = {"time_outs": torch.from_numpy(timeout)}
                ppo.process_env_step(torch.from_numpy(rew), torch.from_numpy(reset), infos)
            ppo.compute_returns(torch.from_numpy(priv))
        ppo.update()
    dt = time.time() - t0
    return n_envs * T * iterations / dt, threads, dt


def comm_report(runner, timer, world, rank_ms):
    """The data-parallel exchange of one iteration (None at world size 1): the per-minibatch
    flat-gradient (+ KL slot) all-reduce and the advantage-statistics all-reduce, each timed with
    HIP events on a sampled subset of the timed region (KernelTimer, this rank), and the per-rank
    spread of the iteration time.  In the one-graph form the gradient all-reduce runs inside the
    replay and is not separable (null)."""
    if world <= 1:
        return None
    alg = runner.alg
    per_it = alg.num_learning_epochs * alg.num_mini_batches
    ar, adv = timer.mean_ms("allreduce"), timer.mean_ms("allreduce_adv_stats")
    sep = timer.count("allreduce") > 0
    total = (per_it * ar if sep else float("nan")) + (adv if timer.count("allreduce_adv_stats") else 0.0)
    nbytes = alg._flat_grad.numel() * alg._flat_grad.element_size() if alg._flat_grad is not None else None
    return {"backend": dist.get_backend(), "update_graph": alg.update_graph,
            "grad_allreduce_bytes": nbytes, "grad_allreduces_per_iteration": per_it,
            "grad_allreduce_ms_mean": round(ar, 4) if sep else None,
            "adv_stats_allreduce_ms_mean": round(adv, 4) if timer.count("allreduce_adv_stats") else None,
            "allreduce_ms_per_iteration": round(total, 4) if sep else None,
            "allreduce_samples": timer.count("allreduce"),
            "timing": f"HIP events on this rank's current stream, 1 in {timer.every} calls of the timed region",
            "rank_ms_per_step": rank_ms}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N ranks with torch.distributed.run (one
    process per GPU, rendezvous on 127.0.0.1) from this parent, which has not touched the GPU, and
    return their exit code.  The ranks see WORLD_SIZE and run the benchmark themselves."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def launch_check(args, world, rank):
    """--launch-check: the multi-rank bookkeeping of a bench run (process group, barriers,
    max-over-ranks time, rank 0's JSON line) with no GPU work, on gloo — the CPU test of the
    launcher (tests/test_bench_launch.py)."""
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.time()
    time.sleep(0.01 * (rank + 1))
    elapsed = time.time() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "value": None, "ms_per_step": round(elapsed * 1e3, 3),
                          "config": {"parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of the run; without WORLD_SIZE in the environment, N > 1 launches "
                         "N ranks itself")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher / rank-bookkeeping check only (no GPU work, gloo)")
    ap.add_argument("--steps", type=int, default=10, help="timed PPO iterations")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--T", type=int, default=24, help="rollout length (num_steps_per_env)")
    ap.add_argument("--cpu-envs", type=int, default=4096, help="CPU baseline sample on all host threads")
    ap.add_argument("--cpu-envs-1core", type=int, default=256, help="CPU baseline sample on one thread")
    ap.add_argument("--cpu-iterations", type=int, default=3, help="PPO iterations of the CPU baseline samples")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gemm-table", action="store_true", help="hipBLASLt default GEMM heuristics")
    ap.add_argument("--terrain", default="plane", choices=["plane", "heightfield"],
                    help="plane = config 2; heightfield = config 3 (2100x2100 generated terrain)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on cuda:0 (with --dist-backend gloo)")
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 5],
                    help="BASELINE.json configs: 2 plane (default), 3 heightfield, 5 push-recovery curriculum "
                         "with 8192 envs/GPU, fp16 observation storage and a bf16 policy")
    args = ap.parse_args()

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus is not None and args.gpus > 1:
        # no launcher: start the ranks from here, before anything initialises the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(world_env or "1")
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to report a {world}-rank run as "
              f"{args.gpus} GPUs", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        launch_check(args, world, rank)
        return

    if args.config == 3:
        args.terrain = "heightfield"
    c5 = args.config == 5
    if c5 and args.envs == 4096:
        args.envs = 8192
    if args.same_device:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    device = f"cuda:{local}"
    # one seed for every rank: the env draws and the action noise are keyed by the global env id
    # (rank r holds envs [r * envs, (r + 1) * envs)), so N ranks run the single N * envs job, split
    torch.manual_seed(5)
    np.random.seed(5)
    from humanoid.algo.ppo import OnPolicyRunner
    from humanoid.utils.blas_tuning import use_tuned_gemms
    tuned = use_tuned_gemms() if not args.no_gemm_table else False
    env = make_env(args.envs, device, seed=5, terrain=args.terrain, push_curriculum=c5, env_offset=rank * args.envs,
                   num_envs_total=world * args.envs)
    runner = OnPolicyRunner(env, train_cfg(args.T, "bf16" if c5 else "fp32", "fp16" if c5 else "fp32"),
                            log_dir=None, device=device)
    timer = KernelTimer(every=int(os.environ.get("HG_TIMER_EVERY", "4")))
    env.kernel_timer = timer
    if world > 1:  # the eager data-parallel all-reduces (gradients + KL per minibatch, advantage stats)
        runner.alg.comm_timer = timer
        runner.alg.storage.comm_timer = timer
    runner.learn(args.warmup, init_at_random_ep_len=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timer.enabled = timer.every > 0
    t0 = time.time()
    runner.learn(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.time() - t0
    timer.enabled = False
    rank_ms = None
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        tmin = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tmin, op=dist.ReduceOp.MIN)
        rank_ms = {"max": round(t.item() / args.steps * 1e3, 3), "min": round(tmin.item() / args.steps * 1e3, 3)}
        elapsed = t.item()
    env_steps = args.envs * args.T * args.steps * world
    value = env_steps / elapsed
    rows = active_rows(env)
    traffic, traffic_src = (pmc_traffic("k_step") if args.envs == 4096 and args.terrain == "plane" and not c5
                            else (None, None))
    ms_step = timer.mean_ms("k_step")
    flops = physics_flops_per_env_step(rows) * args.envs
    achieved_tflops = flops / (ms_step * 1e-3) / 1e12
    roofline = {"kernel": "k_step", "bound": "fp32-valu", "pipe": "fp32 VALU + f32 MFMA (W = Z^T Z); f32 MFMA peak = f32 vector peak",
                "achieved": round(achieved_tflops, 4), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved_tflops / FP32_PEAK_TFLOPS, 6), "traffic": traffic,
                "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": KSTEP_BYTES_PER_ENV * args.envs,
                "hbm_achieved_GBs": round(KSTEP_BYTES_PER_ENV * args.envs / (ms_step * 1e-3) / 1e9, 1),
                "hbm_frac": round(KSTEP_BYTES_PER_ENV * args.envs / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                "valu_issue_util": sq_issue(),
                "valu_issue_source": f"profiles/{PROFILE_DIR}/sq_counters_k_step.json (2 x SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES)",
                "avg_launch_ms": round(ms_step, 4), "launches": timer.count("k_step"),
                "launch_sampling": f"HIP events on 1 in {timer.every} launches of the timed region",
                "flops_per_launch": flops, "active_rows_per_env": round(rows, 2),
                "mfma": mfma_stats(rows, args.envs),
                "k_post_avg_ms": round(timer.mean_ms("k_post"), 4)}
    result = {
        "metric": "env-steps/sec (whole node) at 4096 envs + PPO iters/sec, 1/2/4/8 MI355X",
        "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "ppo_iters_per_sec": round(args.steps / elapsed, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32 physics + bf16 policy" if c5 else "f32", "data": "synthetic",
        "config": {"workload": (f"XBot-L push-recovery curriculum, {args.envs} envs/GPU, fp16 obs storage + bf16 "
                                "policy, PPO 24-step rollout (config 5)" if c5 else
                                "XBot-L flat terrain, 4096 envs/GPU, PPO 24-step rollout (BASELINE configs[1])"
                                if args.terrain == "plane" else
                                "XBot-L heightfield terrain 2100x2100, 4096 envs/GPU, PPO 24-step rollout (config 3)"),
                   "envs_per_gpu": args.envs, "num_steps_per_env": args.T, "parallelism": f"dp{world}",
                   "ppo": "2 epochs x 4 minibatches, actor 705-512-256-128-12, critic 219-768-256-128-1",
                   "update_graph": runner.alg.update_graph,
                   "collectives_per_iteration": runner.alg.collectives_per_update(),
                   "gemm_table": "tuning/tunableop_mi355x_f32.csv" if tuned else None,
                   "gemm": ("f32 operands and accumulation; the large hidden-layer forwards run on the bf16 matrix "
                            "cores as exact three-way bf16 splits of each f32 operand (six partial products, f32 "
                            "accumulation; error per element below torch's f32 GEMM's, tests/test_gpu_gemm.py), "
                            "the other products on f32 MFMA (own kernels) or hipBLASLt f32"
                            if not c5 else "bf16 policy (config 5)")},
        "roofline": roofline,
        "comm": comm_report(runner, timer, world, rank_ms),
        "collection_time_s": round(runner.last_iteration_stats.get("collection_time", float("nan")), 4),
        "learn_time_s": round(runner.last_iteration_stats.get("learn_time", float("nan")), 4),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # config 2 on all host cores for >= 3 iterations (the headline
        # baseline), the same on one core over a smaller sample, and config 1 (4 envs, 1 iteration)
        it = args.cpu_iterations
        v, threads, dt = cpu_baseline(args.cpu_envs, args.T, iterations=it)
        v1, _, dt1 = cpu_baseline(args.cpu_envs_1core, args.T, threads=1, iterations=it)
        vc1, _, dtc1 = cpu_baseline(4, args.T, threads=threads, iterations=1)
        result["cpu_baseline"] = {"value": round(v, 1), "unit": "env-steps/s", "cores": threads, "kind": "port",
                                  "sample": f"{it} PPO iterations, {args.cpu_envs} envs x {args.T} steps, {dt:.1f} s "
                                            f"(oracle physics + numpy env logic + torch-CPU PPO)",
                                  "value_1_core": round(v1, 1),
                                  "sample_1_core": f"{it} PPO iterations, {args.cpu_envs_1core} envs x {args.T} steps, "
                                                   f"{dt1:.1f} s",
                                  "config1": {"value": round(vc1, 1), "unit": "env-steps/s", "cores": threads,
                                              "ppo_iters_per_sec": round(1.0 / dtc1, 3),
                                              "sample": f"BASELINE configs[0]: 1 PPO iteration, 4 envs x {args.T} "
                                                        f"steps, {dtc1:.2f} s"}}
        torch.set_num_threads(threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
