"""Do parallel branches of a captured hipGraph run concurrently on this ROCm?  Times the three
policy MLP forwards (actor / lin-vel / critic at a 24576-row minibatch) captured (a) on one stream
and (b) as three forked branches joined back into the capture stream."""
import torch
import torch.nn as nn
import torch.nn.functional as F

dev = torch.device("cuda:0")
R = 24576


def mlp(i, hs, o):
    L, d = [], i
    for h in hs:
        L += [nn.Linear(d, h), nn.ELU()]
        d = h
    L.append(nn.Linear(d, o))
    return nn.Sequential(*L).to(dev)


nets = [mlp(705, [512, 256, 128], 12), mlp(705, [128, 128], 3), mlp(219, [768, 256, 128], 1)]
xs = [torch.randn(R, 705, device=dev), torch.randn(R, 705, device=dev), torch.randn(R, 219, device=dev)]
outs = [None] * 3


def body(par):
    main = torch.cuda.current_stream()
    if not par:
        for k in range(3):
            outs[k] = nets[k](xs[k])
        return
    for k, s in enumerate(streams):
        s.wait_stream(main)
        with torch.cuda.stream(s):
            outs[k] = nets[k](xs[k])
    for s in streams:
        main.wait_stream(s)


streams = [torch.cuda.Stream() for _ in range(3)]
with torch.no_grad():
    for par in (False, True):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                body(par)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(4):
                body(par)
        torch.cuda.synchronize()
        for _ in range(5):
            g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f"graph {'3 branches' if par else 'sequential'}: {e0.elapsed_time(e1) / 80 * 1e3:.1f} us per 3-net forward")
        # eager
        e0.record()
        for _ in range(80):
            body(par)
        e1.record()
        torch.cuda.synchronize()
        print(f"eager {'3 streams' if par else 'sequential'}: {e0.elapsed_time(e1) / 80 * 1e3:.1f} us per 3-net forward")
