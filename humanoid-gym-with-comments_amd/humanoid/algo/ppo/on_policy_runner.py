"""OnPolicyRunner (humanoid/algo/ppo/on_policy_runner.py:45-322): same constructor, learn() loop
order (T x [act -> env.step -> process_env_step], compute_returns, update), fps formula
(Perf/total_fps = T * num_envs / (collection + learn)), scalar names and checkpoint dict.

Logging backends: TensorBoard's SummaryWriter when importable, otherwise a JSONL scalar writer
(wandb and tensorboard are absent in this image).  Book-keeping reads per-episode stats from
device tensors; the only host syncs per step are the ones the reference also has when log_dir is
set (done-id extraction), so with log_dir=None the rollout is sync-free.
With world_size > 1 (one process per GPU) every rank runs its env shard; rank 0 logs/saves.
"""
import json
import os
import statistics
import time
from collections import deque
from datetime import datetime

import torch
import torch.distributed as dist

from .actor_critic import ActorCritic
from .ppo import PPO


class _JsonlWriter:
    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        self._f = open(os.path.join(log_dir, "scalars.jsonl"), "a")

    def add_scalar(self, tag, value, step):
        self._f.write(json.dumps({"tag": tag, "value": float(value), "step": float(step)}) + "\n")
        self._f.flush()

    def close(self):
        self._f.close()


def _make_writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir=log_dir, flush_secs=10)
    except Exception:
        return _JsonlWriter(log_dir)


def _rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


class OnPolicyRunner:
    def __init__(self, env, train_cfg, log_dir=None, device="cpu"):
        self.cfg = train_cfg["runner"]
        self.alg_cfg = train_cfg["algorithm"]
        self.policy_cfg = train_cfg["policy"]
        self.all_cfg = train_cfg
        self.wandb_run_name = (datetime.now().strftime("%b%d_%H-%M-%S") + "_" + train_cfg["runner"]["experiment_name"]
                               + "_" + train_cfg["runner"]["run_name"])
        self.device = device
        self.env = env
        if hasattr(env, "stable_observations"):
            # PPO copies each observation stack into its rollout storage before the next env.step
            # (hg_rollout_act, or a clone in the non-fused act), so the env may hand out its live
            # window views instead of a fresh copy per step
            env.stable_observations = False
        num_critic_obs = env.num_privileged_obs if env.num_privileged_obs is not None else env.num_obs
        policy_cls = {"ActorCritic": ActorCritic}[self.cfg["policy_class_name"]]
        actor_critic = policy_cls(env.num_obs, num_critic_obs, env.num_actions, **self.policy_cfg).to(self.device)
        alg_cls = {"PPO": PPO}[self.cfg["algorithm_class_name"]]
        self.alg = alg_cls(actor_critic, device=self.device, **self.alg_cfg)
        self.num_steps_per_env = self.cfg["num_steps_per_env"]
        self.save_interval = self.cfg["save_interval"]
        obs_dtype = {"fp32": torch.float32, "fp16": torch.float16}[self.cfg.get("storage_obs_dtype", "fp32")]
        # frame-only actor observation storage when the env stacks frames (one frame per env-step
        # written instead of the whole stack; rollout_storage.py)
        ecfg = getattr(getattr(env, "cfg", None), "env", None)
        fs, w1 = getattr(ecfg, "frame_stack", None), getattr(ecfg, "num_single_obs", None)
        obs_frames = (int(fs), int(w1)) if fs and w1 and int(fs) * int(w1) == env.num_obs else None
        self.alg.init_storage(env.num_envs, self.num_steps_per_env, [env.num_obs], [env.num_privileged_obs],
                              [env.num_actions], obs_dtype=obs_dtype, obs_frames=obs_frames)
        # the action noise is keyed by the global env id of each storage row
        env_cfg = getattr(getattr(env, "cfg", None), "env", None)
        self.alg.row_offset = int(getattr(env_cfg, "env_offset", 0) or 0)
        self.log_dir = log_dir if _rank() == 0 else None
        self.writer = None
        self.tot_timesteps = 0
        self.tot_time = 0
        self.current_learning_iteration = 0
        self.last_iteration_stats = {}
        _, _ = self.env.reset()

    def learn(self, num_learning_iterations, init_at_random_ep_len=False):
        if self.log_dir is not None and self.writer is None:
            self.writer = _make_writer(self.log_dir)
        if init_at_random_ep_len:
            self.env.episode_length_buf = torch.randint_like(self.env.episode_length_buf,
                                                             high=int(self.env.max_episode_length))
        obs = self.env.get_observations()
        privileged_obs = self.env.get_privileged_observations()
        critic_obs = privileged_obs if privileged_obs is not None else obs
        obs, critic_obs = obs.to(self.device), critic_obs.to(self.device)
        self.alg.actor_critic.train()
        ep_infos = []
        rewbuffer = deque(maxlen=100)
        lenbuffer = deque(maxlen=100)
        cur_reward_sum = torch.zeros(self.env.num_envs, dtype=torch.float, device=self.device)
        cur_episode_length = torch.zeros(self.env.num_envs, dtype=torch.float, device=self.device)
        # per-step episode-end records of the rollout, read by the host once per iteration (the
        # reference reads the finished episodes' sums every step: a host wait per policy step)
        T = self.num_steps_per_env
        ep_done = torch.zeros(T, self.env.num_envs, dtype=torch.bool, device=self.device)
        ep_ret = torch.zeros(T, self.env.num_envs, dtype=torch.float, device=self.device)
        ep_len = torch.zeros(T, self.env.num_envs, dtype=torch.float, device=self.device)
        tot_iter = self.current_learning_iteration + num_learning_iterations
        # without a log writer nothing in the loop needs the iteration's numbers on the host: its
        # phase events and loss means are read one iteration later (after the next iteration's
        # work is queued) and at the end, so the GPU never idles at the iteration boundary
        lazy = self.log_dir is None
        pending = None
        for it in range(self.current_learning_iteration, tot_iter):
            if hasattr(self.env, "update_push_curriculum"):
                self.env.update_push_curriculum(it)
            start = time.time()
            on_gpu = self.device != "cpu" and torch.device(self.device).type == "cuda"
            if on_gpu:
                # phase times from HIP events: no host synchronisation between collection and learning
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record()
            sink_ok = hasattr(self.env, "set_rollout_sink") and hasattr(self.alg, "rollout_sink")
            with torch.inference_mode():
                for step in range(self.num_steps_per_env):
                    actions = self.alg.act(obs, critic_obs)
                    if sink_ok:
                        sink = self.alg.rollout_sink()
                        if sink is not None:  # the env's post launch fills the storage slot
                            self.env.set_rollout_sink(*sink)
                    obs, privileged_obs, rewards, dones, infos = self.env.step(actions)
                    critic_obs = privileged_obs if privileged_obs is not None else obs
                    obs, critic_obs = obs.to(self.device), critic_obs.to(self.device)
                    rewards, dones = rewards.to(self.device), dones.to(self.device)
                    self.alg.process_env_step(rewards, dones, infos)
                    if self.log_dir is not None:
                        if "episode" in infos:
                            # hg_sim publishes views into a ring of episode_snapshot_rows launches:
                            # rollouts at least that long keep a copy instead
                            ep = infos["episode"]
                            if self.num_steps_per_env >= getattr(self.env, "episode_snapshot_rows", float("inf")):
                                ep = {k: v.clone() if torch.is_tensor(v) else v for k, v in ep.items()}
                            ep_infos.append(ep)
                        cur_reward_sum += rewards
                        cur_episode_length += 1
                        done = dones.reshape(-1) > 0
                        ep_done[step].copy_(done)
                        ep_ret[step].copy_(cur_reward_sum)
                        ep_len[step].copy_(cur_episode_length)
                        cur_reward_sum.masked_fill_(done, 0)
                        cur_episode_length.masked_fill_(done, 0)
                if on_gpu:
                    ev[1].record()
                stop = time.time()
                collection_time = stop - start
                self.env.course_gain *= self.env.course_ratio
                self.env.course_gain = min(20, self.env.course_gain)
                course_gain = self.env.course_gain
                start = stop
                self.alg.compute_returns(critic_obs)
            if on_gpu and lazy:
                losses = self.alg.update(sync=False)
                ev[2].record()
                # the loss means go to pinned host memory behind the update (a copy queued on the
                # stream, read one iteration later): a plain float() of a device tensor would wait
                # for this iteration's whole update and leave the GPU idle while the host queues
                # the next rollout
                means3 = (losses[0], losses[1], losses[3])
                if all(torch.is_tensor(x) for x in means3):  # device 0-d means (graphed update)
                    dev_means = torch.stack(means3)
                    host_means = torch.empty(dev_means.shape, dtype=torch.float32, pin_memory=True)
                    host_means.copy_(dev_means, non_blocking=True)
                    copied = torch.cuda.Event()
                    copied.record()
                else:  # the eager warm-up update returned host floats
                    host_means, copied = torch.tensor([float(x) for x in means3]), None
                if pending is not None:
                    self._resolve_stats(*pending)
                pending = (ev, host_means, copied)
                ep_infos.clear()
                continue
            mean_value_loss, mean_surrogate_loss, sym_loss, mean_base_lin_vel_loss = self.alg.update()
            stop = time.time()
            learn_time = stop - start
            if on_gpu:
                ev[2].record()
                ev[2].synchronize()
                collection_time = ev[0].elapsed_time(ev[1]) * 1e-3
                learn_time = ev[1].elapsed_time(ev[2]) * 1e-3
            self.last_iteration_stats = dict(collection_time=collection_time, learn_time=learn_time,
                                             value_loss=mean_value_loss, surrogate_loss=mean_surrogate_loss,
                                             lin_vel_loss=mean_base_lin_vel_loss)
            if self.log_dir is not None:
                # the rollout's finished episodes in step order, env order within a step (the
                # order the reference appends them in): one host read per iteration, after the
                # update's own host read
                d, r, ln = ep_done.cpu(), ep_ret.cpu(), ep_len.cpu()
                for t in range(self.num_steps_per_env):
                    ids = d[t].nonzero(as_tuple=False)[:, 0]
                    if ids.numel():
                        rewbuffer.extend(r[t][ids].numpy().tolist())
                        lenbuffer.extend(ln[t][ids].numpy().tolist())
                self.log(locals())
                if it % self.save_interval == 0:
                    self.save(os.path.join(self.log_dir, "model_{}.pt".format(it)))
            ep_infos.clear()
        if pending is not None:
            self._resolve_stats(*pending)
        self.current_learning_iteration += num_learning_iterations
        if self.log_dir is not None:
            self.save(os.path.join(self.log_dir, "model_{}.pt".format(self.current_learning_iteration)))

    def _resolve_stats(self, ev, host_means, copied):
        """last_iteration_stats from an iteration's phase events and its loss means (copied to
        pinned host memory behind that iteration's update; waits for that iteration's end only)."""
        ev[2].synchronize()
        if copied is not None:
            copied.synchronize()
        v, s, lv = [float(x) for x in host_means.tolist()]
        self.last_iteration_stats = dict(collection_time=ev[0].elapsed_time(ev[1]) * 1e-3,
                                         learn_time=ev[1].elapsed_time(ev[2]) * 1e-3,
                                         value_loss=v, surrogate_loss=s, lin_vel_loss=lv)

    def log(self, locs, width=90, pad=45):
        self.tot_timesteps += self.num_steps_per_env * self.env.num_envs
        iteration_time = locs["collection_time"] + locs["learn_time"]
        self.tot_time += iteration_time
        it = locs["it"]
        ep_string = ""
        if locs["ep_infos"]:
            for key in locs["ep_infos"][0]:
                vals = torch.stack([torch.as_tensor(ep[key], device=self.device, dtype=torch.float).reshape(-1)[0]
                                    for ep in locs["ep_infos"]])
                value = vals.mean()
                self.writer.add_scalar("Episode/" + key, value, it)
                ep_string += f"""{f'Mean episode {key}:':>{pad}} {value:.4f}\n"""
        mean_std = self.alg.actor_critic.std.mean()
        fps = int(self.num_steps_per_env * self.env.num_envs / iteration_time)
        w = self.writer
        w.add_scalar("Loss/value_function", locs["mean_value_loss"], it)
        w.add_scalar("Loss/surrogate", locs["mean_surrogate_loss"], it)
        w.add_scalar("Loss/sym_loss", locs["sym_loss"], it)
        w.add_scalar("Train/course_gain", locs["course_gain"], it)
        w.add_scalar("Loss/mean_base_lin_vel_loss", locs["mean_base_lin_vel_loss"], it)
        w.add_scalar("Loss/learning_rate", self.alg.learning_rate, it)
        w.add_scalar("Policy/mean_noise_std", mean_std.item(), it)
        w.add_scalar("Perf/total_fps", fps, it)
        w.add_scalar("Perf/collection time", locs["collection_time"], it)
        w.add_scalar("Perf/learning_time", locs["learn_time"], it)
        if len(locs["rewbuffer"]) > 0:
            w.add_scalar("Train/mean_reward", statistics.mean(locs["rewbuffer"]), it)
            w.add_scalar("Train/mean_episode_length", statistics.mean(locs["lenbuffer"]), it)
            w.add_scalar("Train/mean_reward/time", statistics.mean(locs["rewbuffer"]), self.tot_time)
            w.add_scalar("Train/mean_episode_length/time", statistics.mean(locs["lenbuffer"]), self.tot_time)
        title = f" \033[1m Learning iteration {it}/{self.current_learning_iteration + locs['num_learning_iterations']} \033[0m "
        s = (f"""{'#' * width}\n{title.center(width, ' ')}\n\n"""
             f"""{'Computation:':>{pad}} {fps:.0f} steps/s (collection: {locs['collection_time']:.3f}s, learning {locs['learn_time']:.3f}s)\n"""
             f"""{'Value function loss:':>{pad}} {locs['mean_value_loss']:.4f}\n"""
             f"""{'Surrogate loss:':>{pad}} {locs['mean_surrogate_loss']:.4f}\n"""
             f"""{'Base vel loss:':>{pad}} {locs['mean_base_lin_vel_loss']:.4f}\n"""
             f"""{'Mean action noise std:':>{pad}} {mean_std.item():.2f}\n""")
        if len(locs["rewbuffer"]) > 0:
            s += (f"""{'Mean reward:':>{pad}} {statistics.mean(locs['rewbuffer']):.2f}\n"""
                  f"""{'Mean episode length:':>{pad}} {statistics.mean(locs['lenbuffer']):.2f}\n""")
        s += ep_string
        s += (f"""{'-' * width}\n{'Total timesteps:':>{pad}} {self.tot_timesteps}\n"""
              f"""{'Iteration time:':>{pad}} {iteration_time:.2f}s\n{'Total time:':>{pad}} {self.tot_time:.2f}s\n"""
              f"""{'ETA:':>{pad}} {self.tot_time / (it + 1) * (locs['num_learning_iterations'] - it):.1f}s\n""")
        print(s)

    def save(self, path, infos=None):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        torch.save({"model_state_dict": self.alg.actor_critic.state_dict(),
                    "optimizer_state_dict": self.alg.optimizer.state_dict(),
                    "iter": self.current_learning_iteration, "infos": infos}, path)

    def load(self, path, load_optimizer=True):
        d = torch.load(path, map_location=self.device, weights_only=True)
        self.alg.actor_critic.load_state_dict(d["model_state_dict"])
        if load_optimizer:
            self.alg.optimizer.load_state_dict(d["optimizer_state_dict"])
        self.current_learning_iteration = d["iter"]
        return d["infos"]

    def get_inference_policy(self, device=None):
        self.alg.actor_critic.eval()
        if device is not None:
            self.alg.actor_critic.to(device)
        return self.alg.actor_critic.act_inference

    def get_inference_critic(self, device=None):
        self.alg.actor_critic.eval()
        if device is not None:
            self.alg.actor_critic.to(device)
        return self.alg.actor_critic.evaluate
