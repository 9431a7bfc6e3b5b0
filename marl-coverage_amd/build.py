"""Build libmarlcov.so for gfx950 with hipcc (no cmake, no JIT cache: the .so
is written in-tree so it travels with the repo to the GPU box)."""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmarlcov.so")
ARCH = os.environ.get("MARLCOV_ARCH", "gfx950")

# No -ffast-math / -ffp-contract=fast: the lidar march and reward assembly
# must keep the reference's IEEE float64 adds and correctly rounded division.
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-function"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def deps():
    return sources() + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(ROOT, "include", "marlcov.h")]


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(p) <= t for p in deps())


def build(force=False, verbose=False):
    if not force and up_to_date():
        return OUT
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    cmd = [hipcc, *FLAGS, "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-o", OUT + ".tmp", *sources()]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
