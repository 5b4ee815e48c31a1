"""BaseTask: the env-side buffer/API contract of the reference
(humanoid/envs/base/base_task.py:43-152), without Isaac Gym.

The reference allocates obs/rew/reset/episode-length buffers here and creates the PhysX sim.
In this build the buffers live inside the hg_sim device arena (SoA, caller-allocated) and are
exposed as zero-copy torch views by the subclass's create_sim(); BaseTask keeps the sizes,
device handling and the public methods.  Viewer/camera code is out of scope (headless only).
"""
import torch


class BaseTask:
    def __init__(self, cfg, sim_params, physics_engine, sim_device, headless):
        self.sim_params = sim_params
        self.physics_engine = physics_engine
        self.sim_device = sim_device
        self.headless = True
        dev = torch.device(sim_device)
        if dev.type != "cuda":
            raise RuntimeError(
                f"XBot-L env runs on the hg_sim HIP kernels and needs a ROCm GPU device (got {sim_device!r}); "
                "there is no CPU simulation backend on the product path")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.sim_device_id = dev.index
        self.graphics_device_id = -1
        self.num_envs = cfg.env.num_envs
        self.num_obs = cfg.env.num_observations
        self.num_privileged_obs = cfg.env.num_privileged_obs
        self.num_actions = cfg.env.num_actions
        self.extras = {}
        self.viewer = None
        self.enable_viewer_sync = False
        self.create_sim()

    def get_observations(self):
        return self.obs_buf

    def get_privileged_observations(self):
        return self.privileged_obs_buf

    def reset_idx(self, env_ids):
        raise NotImplementedError

    def reset(self):
        """Reset all robots (base_task.py:144-149): reset_idx(all) then one zero-action step."""
        self.reset_idx(torch.arange(self.num_envs, device=self.device))
        obs, privileged_obs, _, _, _ = self.step(
            torch.zeros(self.num_envs, self.num_actions, device=self.device, requires_grad=False))
        return obs, privileged_obs

    def step(self, actions):
        raise NotImplementedError

    def render(self, sync_frame_time=True):
        return None
