"""Per-map phase timing of the dist_reward full-transform kernel at C5 steady
state (diagnostic build, -DMC_DIST_STAMPS; csrc/mc_dist.hip DSTAMP).

    python tools/dist_stamps.py [--envs 8192] [--warmup 600] [--build-only]

Runs C5 to step `warmup`, steps once more with the stamp buffer attached and
prints, for the maps that step listed, the staging / main-strip / cache-pass
cycles (median, p90, max) split by path (cache fast path or full transform)
and how the cache list was rebuilt.  Stamps perturb the schedule: read shares.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = os.path.join(ROOT, "marl-coverage_amd")
LIB = os.path.join(PKG, "libmarlcov_dstamps.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--warmup", type=int, default=600)  # 5: the early phase after a reset
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    if args.build_only:
        sys.path.insert(0, PKG)
        import build as mcbuild
        mcbuild.build(extra_flags=["-DMC_DIST_STAMPS"], out=LIB)
        return
    os.environ["MARLCOV_LIB"] = LIB
    import numpy as np
    import torch
    import marlcov
    from marlcov import _lib
    import bench

    c = bench.CONFIGS["c5"]
    cfg = dict(bench.BASE, numrobot=c["numrobot"], sensor_config=c["sensor_config"], maxsteps=2000,
               **c.get("extra", {}))
    B = args.envs
    env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=512, length=512, prob_obst=0.1, seed=1000),
                                   seed=1, auto_reset=True)
    env.reset()
    for t in range(args.warmup):
        env.step(env.random_actions(7, t))
    st = torch.zeros((B * 16 + 24576,), dtype=torch.int64, device=env.device)  # + per-part records
    _lib.check(env.lib.mc_debug_stamps(env._h, st.data_ptr()), "stamps")
    env.step(env.random_actions(7, args.warmup))
    torch.cuda.synchronize()
    listed = int(env.get_state(_lib.FIELD_DIST_LISTED).item())
    served = int(env.get_state(_lib.FIELD_DIST_CACHED).item())
    allst = st.cpu().numpy().reshape(-1).astype(np.uint64)
    s = allst[:B * 16]
    s = s[s != 0]
    parts = allst[B * 16:B * 16 + 4096]
    parts = parts[parts != 0]
    t0 = allst[B * 16 + 12288:B * 16 + 16384].astype(np.int64)
    t1 = allst[B * 16 + 16384:B * 16 + 20480].astype(np.int64)
    tk = allst[B * 16 + 20480:B * 16 + 24576].astype(np.int64)
    live = t0 != 0
    sub = allst[B * 16 + 8192:B * 16 + 12288]
    sub = sub[sub != 0]
    merged_tot = allst[B * 16 + 4096:B * 16 + 8192]
    merged_tot = (merged_tot[merged_tot != 0] & np.uint64(0xFFFFFF)).astype(np.int64) * 16
    print(f"step {args.warmup + 1}: listed {listed}, cache served {served}, stamped {len(s)}")
    fast = (s >> np.uint64(48)) & np.uint64(1)
    kept = (s >> np.uint64(49)) & np.uint64(1)
    second = (s >> np.uint64(50)) & np.uint64(1)
    ph = [((s >> np.uint64(16 * i)) & np.uint64(0xFFFF)).astype(np.int64) * 16 for i in range(3)]
    ph.insert(0, (s >> np.uint64(51)).astype(np.int64) * 64)  # the fast-path attempt (part of stage)
    part = (s >> np.uint64(52)) & np.uint64(1)  # a split map's part (mode 2; mode 3 does not stamp)
    fast = fast & (np.uint64(1) - part)
    for name, m in (("split part", part == 1), ("fast path", fast == 1), ("full, one-pass list", (fast == 0) & (kept == 1)),
                    ("full, second pass", (fast == 0) & (second == 1)),
                    ("full, no cache", (fast == 0) & (kept == 0) & (second == 0))):
        if not m.any():
            print(f"  {name:22s} n=0")
            continue
        # dist_fast_kernel's served maps: the try's staging, span + cell
        # search, target search; the transform kernels: fast-path attempt, stage,
        # strips, cache pass
        labs = (("", "stage", "cells", "targets") if name == "fast path" else
                ("", "stage", "strips", "publish") if name == "split part" else ("fast try", "stage", "strips", "cache"))
        row = "  ".join(f"{lab} med {np.median(p[m]):8.0f} p90 {np.percentile(p[m], 90):8.0f} max {p[m].max():8d}"
                        for lab, p in zip(labs, ph) if lab)
        print(f"  {name:22s} n={m.sum():5d}  {row}")
    if len(parts):
        f = [((parts >> np.uint64(16 * i)) & np.uint64(0xFFFF)).astype(np.int64) * 16 for i in range(3)]
        nrun = ((parts >> np.uint64(48)) & np.uint64(63)).astype(np.int64)
        S = ((parts >> np.uint64(54)) & np.uint64(15)).astype(np.int64)
        tot = f[0] + f[1] + f[2]
        print(f"  parts: n={len(parts)}  S values {sorted(set(S.tolist()))}  part total med {np.median(tot):.0f} "
              f"p90 {np.percentile(tot, 90):.0f} max {tot.max()}")
        for k in sorted(set(nrun.tolist())):
            m = nrun == k
            print(f"    strips run {k:2d}: n={m.sum():4d}  stage med {np.median(f[0][m]):7.0f}  strips med "
                  f"{np.median(f[1][m]):7.0f} max {f[1][m].max():7d}  publish med {np.median(f[2][m]):7.0f} "
                  f"max {f[2][m].max():7d}")
        if len(sub):
            g = [((sub >> np.uint64(16 * i)) & np.uint64(0xFFFF)).astype(np.int64) * 16 for i in range(3)]
            print("    stage split: " + "  ".join(f"{lab} med {np.median(x):7.0f} p90 {np.percentile(x, 90):7.0f}"
                                              for lab, x in zip(("loads+transpose", "barrier", "extend rows"), g)))
        if live.any():
            base = tk[live].min()
            print(f"    timeline (cycles from the first part's start): workgroup start med "
                  f"{np.median(tk[live] - base):.0f} max {(tk[live] - base).max()}; item start med "
                  f"{np.median(t0[live] - base):.0f} max {(t0[live] - base).max()}; part end med "
                  f"{np.median(t1[live] - base):.0f} p90 {np.percentile(t1[live] - base, 90):.0f} max "
                  f"{(t1[live] - base).max()}")
        if len(merged_tot):
            print(f"  merged parts (start -> done): n={len(merged_tot)} med {np.median(merged_tot):.0f} "
                  f"p90 {np.percentile(merged_tot, 90):.0f} max {merged_tot.max()}")


if __name__ == "__main__":
    main()
