"""Fixed cost of bench.py's timed region (C2, back-to-back stream launches).

    python tools/sync_probe.py [auto|spin|yield|blocking]

Sets the HIP device schedule flag (before the device is initialised), then
times K launches between synchronizes for K in (1, 20, 200), 10 reps each,
and prints per K the median wall time, the HIP-event time, the host enqueue
time and the wall - events gap (launch latency + synchronize wake-up).
"""
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

FLAGS = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "auto"
    hip = ctypes.CDLL("libamdhip64.so")
    if mode != "auto":
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(FLAGS[mode]))
        print(f"hipSetDeviceFlags({mode}) rc={rc}", flush=True)
    import bench
    import marlcov

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = bench.CONFIGS["c2"]
    B, N = c["envs"], c["numrobot"]
    cfg = dict(bench.BASE, numrobot=N, sensor_config=c["sensor_config"], allow_even_beams=True)
    env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=128, length=128, prob_obst=0.1, seed=1000,
                                                    num_grids=B), device=dev, seed=1, auto_reset=True)
    env.reset()
    acts = torch.randint(0, 4, (64, B, N), dtype=torch.uint8, device=dev)
    rp, dp, op = env.reward.data_ptr(), env.done.data_ptr(), env.obs.data_ptr()
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    for i in range(30):
        env.step_raw(acts[i % 64].data_ptr(), rp, dp, op, sp)
    torch.cuda.synchronize(dev)
    # an empty synchronize
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    print(f"{mode}: empty synchronize {1e6 * statistics.median(ts):.1f} us", flush=True)
    for K in (1, 20, 200):
        walls, evs, enq = [], [], []
        for rep in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            e0.record(stream)
            for i in range(K):
                env.step_raw(acts[i % 64].data_ptr(), rp, dp, op, sp)
            e1.record(stream)
            t1 = time.perf_counter()
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            walls.append(t2 - t0)
            enq.append(t1 - t0)
            evs.append(e0.elapsed_time(e1) * 1e-3)
        w, e, q = (statistics.median(x) * 1e6 for x in (walls, evs, enq))
        print(f"{mode}: K={K:3d} wall {w:8.1f} us  events {e:8.1f} us  enqueue {q:8.1f} us  "
              f"gap {w - e:6.1f} us  ({w / K:6.2f} us/step wall)", flush=True)


if __name__ == "__main__":
    main()
