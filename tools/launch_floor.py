"""Back-to-back launch cadence of a trivial kernel on one stream (the floor
under any per-step kernel time): events around K launches / K, issued from
Python (host-bound) and replayed from a hipGraph (GPU-side gap)."""
import torch

x = torch.zeros(1, device="cuda")
y = torch.zeros(1 << 20, device="cuda")
K = 500
for name, fn in [("tiny add_ (1 elem)", lambda: x.add_(1)), ("fill 4 MB", lambda: y.fill_(1.0))]:
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: stream {e0.elapsed_time(e1) / K * 1e3:.2f} us per launch")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(K):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: graph {e0.elapsed_time(e1) / K * 1e3:.2f} us per launch")
