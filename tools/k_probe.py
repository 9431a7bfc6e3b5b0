"""Where does the fixed cost of a short timed region go? (C2, hipGraph replay)

Times K-step graph replays like bench.py does, in variants: a fresh graph's
first replay, the same after hipGraphUpload, and a second replay.  Prints one
line per variant: host wall us/step and HIP-event us/step.
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import marlcov  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]


def main():
    dev = torch.device("cuda", 0)
    c = bench.CONFIGS["c2"]
    B, N = c["envs"], c["numrobot"]
    cfg = dict(bench.BASE, numrobot=N, sensor_config=c["sensor_config"], allow_even_beams=True)
    env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=128, length=128, prob_obst=0.1, seed=1000,
                                                    num_grids=B), device=dev, seed=1, auto_reset=True)
    env.reset()
    acts = torch.randint(0, 4, (4000, B, N), dtype=torch.uint8, device=dev)
    rp, dp, op = env.reward.data_ptr(), env.done.data_ptr(), env.obs.data_ptr()
    stream = torch.cuda.current_stream(dev)
    nxt = [0]

    def eager(n):
        for _ in range(n):
            env.step_raw(acts[nxt[0]].data_ptr(), rp, dp, op, stream.cuda_stream)
            nxt[0] += 1

    def capture(K):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cs = torch.cuda.current_stream(dev).cuda_stream
            for _ in range(K):
                env.step_raw(acts[nxt[0]].data_ptr(), rp, dp, op, cs)
                nxt[0] += 1
        torch.cuda.synchronize(dev)
        return g

    def timed(g, K, tag):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        e0.record(stream)
        g.replay()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        print(f"{tag:40s} K={K:4d} wall {1e6 * (t1 - t0) / K:7.2f} us/step  events "
              f"{1e3 * e0.elapsed_time(e1) / K:7.2f} us/step", flush=True)

    eager(5)
    torch.cuda.synchronize(dev)
    for K in (20, 200):
        g = capture(K)
        timed(g, K, "fresh graph, first replay")
        timed(g, K, "same graph, second replay")
        g2 = capture(K)
        rc = hip.hipGraphUpload(ctypes.c_void_p(g2.raw_cuda_graph_exec()), ctypes.c_void_p(stream.cuda_stream))
        torch.cuda.synchronize(dev)
        timed(g2, K, f"fresh graph + hipGraphUpload (rc {rc})")
        eager(3)
        torch.cuda.synchronize(dev)
        timed(g2, K, "uploaded graph after 3 eager steps")
    # eager per-step
    for K in (20, 200):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        eager(K)
        torch.cuda.synchronize(dev)
        print(f"{'eager':40s} K={K:4d} wall {1e6 * (time.perf_counter() - t0) / K:7.2f} us/step")
    env.check()


if __name__ == "__main__":
    main()
