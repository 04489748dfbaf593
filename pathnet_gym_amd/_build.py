"""Build the HIP kernel library for gfx950 (in-tree, no JIT cache).

``python -m pathnet_gym_amd._build`` compiles every ``csrc/*.hip`` with hipcc
(``--offload-arch=gfx950``) into ``pathnet_gym_amd/_hip/libpathnet_hip.so``.
The library has a plain C ABI (raw device pointers + hipStream_t) and is
loaded with ctypes after torch, so it shares torch's HIP runtime
(libamdhip64.so.7).  Objects are rebuilt only when a source or header is
newer than the object.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.join(ROOT, "pathnet_gym_amd", "_hip")
LIB = os.path.join(OUT_DIR, "libpathnet_hip.so")
ARCH = os.environ.get("PATHNET_HIP_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result"]


def _needs(obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, jobs: int = 0) -> str:
    os.makedirs(OUT_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(OUT_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if _needs(o, [s] + headers):
            todo.append((s, o))

    def comp(so):
        s, o = so
        cmd = [HIPCC] + FLAGS + ["-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {s}:\n{r.stderr}")
        return o

    n = jobs or min(8, max(1, (os.cpu_count() or 2)))
    n = min(n, 16)
    with cf.ThreadPoolExecutor(n) as ex:
        list(ex.map(comp, todo))
    if todo or not os.path.exists(LIB):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
