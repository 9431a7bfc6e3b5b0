"""Microbenchmark of the full distance transform: one C5 reset runs it on
every map (all M unknown).  Used under rocprofv3 (kernel trace / PMC)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import marlcov
from bench import BASE, CONFIGS

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
c = CONFIGS["c5"]
cfg = dict(BASE, numrobot=c["numrobot"], sensor_config=c["sensor_config"], maxsteps=2000, **c["extra"])
env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=512, length=512, prob_obst=0.1, seed=1000, num_grids=B),
                               device="cuda:0", seed=1, auto_reset=True)
for _ in range(3):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    env.reset()
    torch.cuda.synchronize(); t1 = time.perf_counter()
    print(f"reset of {B} envs ({B * 16} full transforms): {(t1 - t0) * 1e3:.2f} ms", flush=True)
env.check()
