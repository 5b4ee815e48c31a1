"""The actor + lin-vel forward/backward at the minibatch size (24576 rows) as two separate fused MLP
calls vs hg_mlp.mlp_pair_forward (stacked first layer), timed with HIP events (MODE=sep|pair|both)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
import torch  # noqa: E402

from humanoid.algo.ppo import ActorCritic, hg_mlp  # noqa: E402
from humanoid.utils.blas_tuning import use_tuned_gemms  # noqa: E402

use_tuned_gemms()
torch.manual_seed(0)
ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
                 base_lin_vel_hidden_dims=[128, 128]).cuda()
rows = 24576
x = torch.randn(rows, 705, device="cuda:0")
params = [*ac.actor.parameters(), *ac.base_lin_vel.parameters()]
ga, gb = torch.randn(rows, 12, device="cuda:0"), torch.randn(rows, 3, device="cuda:0")


def sep():
    with hg_mlp.image_scope([(ac.actor, rows), (ac.base_lin_vel, rows)], x.device):
        ya, yb = hg_mlp.mlp_forward(ac.actor, x), hg_mlp.mlp_forward(ac.base_lin_vel, x)
    torch.autograd.grad((ya, yb), params, (ga, gb))


def pair():
    with hg_mlp.image_scope([(ac.actor, rows), (ac.base_lin_vel, rows)], x.device,
                            pairs=[(ac.actor, ac.base_lin_vel, rows)]):
        ya, yb = hg_mlp.mlp_pair_forward(ac.actor, ac.base_lin_vel, x)
    torch.autograd.grad((ya, yb), params, (ga, gb))


for name, fn in (("sep", sep), ("pair", pair)):
    if os.environ.get("MODE", "both") not in ("both", name):
        continue
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us per forward + backward", flush=True)
