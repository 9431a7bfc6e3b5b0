"""Build libmarlcov.so for gfx950 with hipcc (no cmake, no JIT cache: the .so
is written in-tree so it travels with the repo to the GPU box).

Each csrc/*.hip is compiled to its own object in parallel (objects under
build/, rebuilt when the source or any header is newer), then linked."""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
OUT = os.path.join(HERE, "libmarlcov.so")
ARCH = os.environ.get("MARLCOV_ARCH", "gfx950")

# No -ffast-math, and contraction explicitly off (hipcc's device default is
# -ffp-contract=fast-honor-pragmas, which may fuse a multiply and an add into
# an FMA): the lidar march, the reward assembly and the float32 distance
# terms must keep the reference's separately rounded IEEE operations
# (NumPy never fuses).  The minimap's bilinear weights additionally use
# __dmul_rn / __dadd_rn (mc_minimap.hip), which no flag can fuse.
CFLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
          "-Wno-unused-function"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(ROOT, "include", "marlcov.h")]


def deps():
    return sources() + headers()


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(p) <= t for p in deps())


def _obj(src, extra):
    tag = ("-" + "_".join(f.strip("-").replace("=", "") for f in extra)) if extra else ""
    return os.path.join(OBJ, os.path.basename(src)[:-4] + tag + ".o")


def build(force=False, verbose=False, extra_flags=(), out=None):
    """Compile (changed) objects in parallel and link; `extra_flags` (e.g.
    ['-DMC_STAMPS']) build a diagnostic variant into `out`."""
    extra = list(extra_flags)
    out = out or OUT
    if not force and not extra and out == OUT and up_to_date():
        return out
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    os.makedirs(OBJ, exist_ok=True)
    hdr_t = max(os.path.getmtime(h) for h in headers())
    inc = ["-I", os.path.join(ROOT, "include"), "-I", CSRC]

    def compile_one(src):
        obj = _obj(src, extra)
        if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_t):
            return obj
        cmd = [hipcc, *CFLAGS, *extra, *inc, "-c", "-o", obj + ".tmp", src]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
        return obj

    jobs = min(len(sources()), max(1, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, sources()))
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp", *objs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
