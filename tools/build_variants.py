"""Build diagnostic variants of libmarlcov.so for A/B runs on the GPU box.

    python tools/build_variants.py NAME:FLAGS [NAME:FLAGS ...]
e.g.  stamps:-DMC_STAMPS  base:   -> marl-coverage_amd/libmarlcov_v_<NAME>.so
Select one with MARLCOV_LIB=<path> (marlcov/_lib.py).
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "marl-coverage_amd")


def build(spec):
    name, _, flags = spec.partition(":")
    out = os.path.join(PKG, f"libmarlcov_v_{name}.so")
    srcs = sorted(glob.glob(os.path.join(PKG, "csrc", "*.hip")))
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-ffp-contract=off", "-shared",
           *flags.split(), "-I", os.path.join(ROOT, "include"), "-I", os.path.join(PKG, "csrc"),
           "-o", out, *srcs]
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    with ThreadPoolExecutor(4) as ex:
        for p in ex.map(build, sys.argv[1:]):
            print(p)
