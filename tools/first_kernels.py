"""Per-launch HIP-event durations of the first timed launches after a
synchronize (C2, the bench's short form: 5 warmup steps, 20 timed), and the
same right after a busy stream, to see whether the first launches of a
short timed region run slower (cold clocks or caches)."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import marlcov  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    c = bench.CONFIGS["c2"]
    B, N = c["envs"], c["numrobot"]
    cfg = dict(bench.BASE, numrobot=N, sensor_config=c["sensor_config"], allow_even_beams=True)
    env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=128, length=128, prob_obst=0.1, seed=1000,
                                                    num_grids=B), device=dev, seed=1, auto_reset=True)
    env.reset()
    acts = torch.randint(0, 4, (64, B, N), dtype=torch.uint8, device=dev)
    rp, dp, op = env.reward.data_ptr(), env.done.data_ptr(), env.obs.data_ptr()
    sp = torch.cuda.current_stream(dev).cuda_stream
    st = torch.cuda.current_stream(dev)
    for rep in range(3):
        for i in range(5):
            env.step_raw(acts[i].data_ptr(), rp, dp, op, sp)
        torch.cuda.synchronize(dev)
        env.check()
        for pause_ms in (0.0, 1.0):
            if pause_ms:
                time.sleep(pause_ms * 1e-3)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
            torch.cuda.synchronize(dev)
            ev[0].record(st)
            for i in range(20):
                env.step_raw(acts[i].data_ptr(), rp, dp, op, sp)
                ev[i + 1].record(st)
            torch.cuda.synchronize(dev)
            d = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(20)]
            print(f"rep {rep} pause {pause_ms} ms: first 5 " + " ".join(f"{x:.2f}" for x in d[:5]) +
                  f" | median of rest {statistics.median(d[5:]):.2f} us", flush=True)


if __name__ == "__main__":
    main()
