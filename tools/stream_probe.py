"""C2 throughput with the 4096-env batch split into S shards on S HIP streams
(each shard's launches stream-ordered, shards independent: no cross-stream
sync inside the timed region), against one 4096-env handle on one stream."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import marlcov  # noqa: E402


def run(S, total=4096, K=200, W=20, reps=3):
    dev = torch.device("cuda", 0)
    c = bench.CONFIGS["c2"]
    N = c["numrobot"]
    cfg = dict(bench.BASE, numrobot=N, sensor_config=c["sensor_config"], allow_even_beams=True)
    B = total // S
    envs, streams, acts = [], [], []
    for k in range(S):
        st = torch.cuda.Stream(dev)
        with torch.cuda.stream(st):
            env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=128, length=128, prob_obst=0.1,
                                                            seed=1000 + k, num_grids=B),
                                           device=dev, seed=1 + k, auto_reset=True)
            env.reset()
            a = torch.randint(0, 4, (W + K, B, N), dtype=torch.uint8, device=dev)
        envs.append(env)
        streams.append(st)
        acts.append(a)
    torch.cuda.synchronize(dev)
    ptrs = [(e.reward.data_ptr(), e.done.data_ptr(), e.obs.data_ptr()) for e in envs]
    sps = [s.cuda_stream for s in streams]
    for i in range(W):
        for k in range(S):
            envs[k].step_raw(acts[k][i].data_ptr(), *ptrs[k], sps[k])
    torch.cuda.synchronize(dev)
    out = []
    for rep in range(reps):
        for Kt in (K, 20):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for i in range(Kt):
                for k in range(S):
                    envs[k].step_raw(acts[k][W + (i % K)].data_ptr(), *ptrs[k], sps[k])
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            out.append((Kt, total * Kt / dt / 1e6, dt / Kt * 1e6))
    for e in envs:
        e.check()
    return out


if __name__ == "__main__":
    for S in (1, 2, 4, 1, 2, 4):
        for Kt, rate, us in run(S):
            print(f"S={S} K={Kt}: {rate:.1f} M env-steps/s, {us:.2f} us/step", flush=True)
