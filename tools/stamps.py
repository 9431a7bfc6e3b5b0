"""Phase timing of the env kernel from s_memtime stamps (diagnostic build).

    python tools/stamps.py [--envs 4096] [--config c2]
Builds marl-coverage_amd/libmarlcov_stamps.so with -DMC_STAMPS and prints, per
phase, the median / p90 / max cycles over all envs of the last step, plus the
spread of wave start times.  Stamps perturb the schedule: read shares, not
absolute kernel time.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = os.path.join(ROOT, "marl-coverage_amd")
LIB = os.path.join(PKG, "libmarlcov_stamps.so")
PHASES = ["rt1 pos/act/scalars", "rt2 stage", "moves", "sense", "merge", "reward",
          "store", "(reset)", "obs", "adj+drain"]


def build():
    sys.path.insert(0, PKG)
    import build as mcbuild  # marl-coverage_amd/build.py
    mcbuild.build(extra_flags=["-DMC_STAMPS"], out=LIB)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--lib", default=LIB, help="a stamped library (tools/build_variants.py NAME:-DMC_STAMPS ...)")
    args = ap.parse_args()
    if args.lib == LIB and (args.build_only or not os.path.exists(LIB)):
        build()
        if args.build_only:
            return
    os.environ["MARLCOV_LIB"] = args.lib
    print("library:", os.environ["MARLCOV_LIB"])
    import numpy as np
    import torch
    import marlcov
    from marlcov import _lib
    import bench

    c = bench.CONFIGS[args.config]
    cfg = dict(bench.BASE, numrobot=c["numrobot"], sensor_config=c["sensor_config"], allow_even_beams=True,
               **c.get("extra", {}))
    B = args.envs
    env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=c["width"], length=c["width"], prob_obst=0.1, seed=1000),
                                   seed=1, auto_reset=True)
    print("kernel:", env.kernel_variant())
    st = torch.zeros((B, 16), dtype=torch.int64, device=env.device)
    _lib.check(env.lib.mc_debug_stamps(env._h, st.data_ptr()), "stamps")
    env.reset()
    for t in range(args.steps):
        a = torch.randint(0, 4, (B, env.num_agents), dtype=torch.uint8, device=env.device)
        env.step(a)
    torch.cuda.synchronize()
    s = st.cpu().numpy().astype(np.int64)
    s = s[s[:, 0] > 0]  # one stamp row per workgroup (first env slot)
    t0 = s[:, 0].min()
    print(f"envs={B}  wave start spread (cycles): median {np.median(s[:,0]-t0):.0f}  max {(s[:,0]-t0).max()}")
    print(f"kernel span (first start -> last end): {s[:,10].max()-t0} cycles")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    acts = torch.randint(0, 4, (20, B, env.num_agents), dtype=torch.uint8, device=env.device)
    ev0.record()
    for t in range(20):
        env.step(acts[t])
    ev1.record()
    torch.cuda.synchronize()
    print(f"eager step (stamped build): {ev0.elapsed_time(ev1) / 20 * 1000:.2f} us")
    order = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 7), (7, 8), (8, 9), (9, 10)]
    for (i, j), name in zip(order, PHASES):
        ok = (s[:, i] > 0) & (s[:, j] > 0)
        if not ok.any():
            print(f"  {name:22s} (no samples)")
            continue
        d = s[ok, j] - s[ok, i]
        print(f"  {name:22s} median {np.median(d):8.0f}  p90 {np.percentile(d,90):8.0f}  max {d.max():8d}  n={ok.sum()}")
    for (i, j), name in [((1, 11), "stage: issue"), ((1, 15), "stage: load issue (early moves)"),
                         ((15, 11), "stage: moves (early moves)"), ((11, 12), "stage: wait"), ((12, 2), "stage: lds"),
                         ((3, 13), "sense: march"), ((13, 4), "sense: gather"),
                         ((4, 14), "merge: mask wait"), ((14, 5), "merge: work+barrier")]:
        ok = (s[:, i] > 0) & (s[:, j] > 0)
        if ok.any():
            d = s[ok, j] - s[ok, i]
            print(f"    {name:20s} median {np.median(d):8.0f}  p90 {np.percentile(d,90):8.0f}")
    tot = s[:, 10] - s[:, 0]
    print(f"  {'whole wave':22s} median {np.median(tot):8.0f}  p90 {np.percentile(tot,90):8.0f}  max {tot.max():8d}")


if __name__ == "__main__":
    main()
