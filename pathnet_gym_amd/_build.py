"""Build the HIP kernel library for gfx950 (in-tree, no JIT cache).

``python -m pathnet_gym_amd._build`` compiles every ``csrc/*.hip`` with hipcc
(``--offload-arch=gfx950``) into ``pathnet_gym_amd/_hip/libpathnet_hip.so``.
The library has a plain C ABI (raw device pointers + hipStream_t) and is
loaded with ctypes after torch, so it shares torch's HIP runtime
(libamdhip64.so.7).  An object is rebuilt when the SHA-256 of its source,
the shared headers and the compile flags differs from the stamp written next
to it (``<obj>.sha``); the library is relinked when the combined stamp of
its objects changes.  The stamp also records the SHA-256 of the built file itself,
which is re-verified before the file is trusted: an object or library that does not
match its stamp (e.g. a stale file shipped next to a fresh stamp) is rebuilt.  File
mtimes are never trusted: a snapshot pushed to a GPU box with skewed mtimes still
rebuilds exactly what changed.

Reproducible: every object is compiled with an explicit ``-cuid=<source name>`` from
relative paths, so the bytes depend only on the sources, the flags and the compiler --
not on the checkout path or the output file name (hipcc otherwise derives the
compilation-unit id from them).  ``python -m pathnet_gym_amd._build --verify`` cold-builds
every source into a scratch directory and compares each object and the library with the
shipped ones byte for byte (bench.py runs it on the GPU box, in the background).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
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
REPRO = "cuid=<source name>, relative paths"      # part of every object's stamp (see _compile)


def _digest(paths, extra=()) -> str:
    h = hashlib.sha256()
    for x in extra:
        h.update(str(x).encode())
        h.update(b"\0")
    for p in paths:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _file_sha(path) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def _stamp(path):
    """(input digest, sha256 of the built file) recorded next to ``path``."""
    try:
        with open(path + ".sha") as f:
            lines = f.read().split()
    except OSError:
        return "", ""
    return (lines + ["", ""])[0], (lines + ["", ""])[1]


def _write_stamp(path, digest):
    with open(path + ".sha", "w") as f:
        f.write(digest + "\n" + _file_sha(path) + "\n")


def _needs(obj, digest) -> bool:
    if not os.path.exists(obj):
        return True
    d, fsha = _stamp(obj)
    return d != digest or fsha != _file_sha(obj)


LAST = {"compiled": [], "relinked": False}       # what the last build() call in this process did


def source_digest() -> str:
    """SHA-256 over every csrc/*.hip and csrc/*.h (names + contents), computed from the files on disk now."""
    return _digest(sorted(glob.glob(os.path.join(CSRC, "*.hip"))) + sorted(glob.glob(os.path.join(CSRC, "*.h"))))


def build_info(lib: str = LIB) -> dict:
    """Provenance of the loaded library for result records: the digest of the sources on disk, the SHA-256 of the
    library file, and which objects this process compiled (an object or library whose stamp does not match its
    sources, flags or own bytes is rebuilt by build(), so the library always derives from these sources)."""
    return {"sources_sha256": source_digest()[:16], "lib_sha256": _file_sha(lib)[:16],
            "compiled_here": [os.path.basename(o) for o in LAST["compiled"]], "relinked_here": LAST["relinked"],
            "arch": ARCH}


def build(verbose: bool = False, jobs: int = 0) -> str:
    """Compile what is stale and relink.  Ranks of one job that call this together (bench.py under torchrun) are
    serialised by an exclusive lock on the output directory: the first compiles, the others then find it current."""
    os.makedirs(OUT_DIR, exist_ok=True)
    import fcntl
    with open(os.path.join(OUT_DIR, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            return _build_locked(verbose, jobs)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_locked(verbose: bool, jobs: int) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = sorted(glob.glob(os.path.join(CSRC, "*.h")))
    objs = []
    todo = []
    digests = []
    for s in srcs:
        o = os.path.join(OUT_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        d = _digest([s] + headers, [HIPCC] + FLAGS + [REPRO])
        digests.append(d)
        if _needs(o, d):
            todo.append((s, o, d))

    def comp(sod):
        s, o, d = sod
        _compile(s, o, verbose)
        _write_stamp(o, d)
        return o

    with cf.ThreadPoolExecutor(_jobs(jobs)) as ex:
        list(ex.map(comp, todo))
    LAST["compiled"] = [o for _, o, _ in todo]
    LAST["relinked"] = False
    lib_digest = hashlib.sha256("".join(digests).encode()).hexdigest()
    if todo or _needs(LIB, lib_digest):
        LAST["relinked"] = True
        _link(objs, LIB)
        _write_stamp(LIB, lib_digest)
    return LIB


def _jobs(jobs: int) -> int:
    n = jobs or min(8, max(1, (os.cpu_count() or 2)))
    return min(n, 16)


def _compile(src: str, obj: str, verbose: bool = False):
    """One object, reproducibly: relative paths from the repo root and an explicit compilation-unit id."""
    cuid = os.path.basename(src).replace(".", "_")
    cmd = [HIPCC] + FLAGS + [f"-cuid={cuid}", "-c", os.path.relpath(src, ROOT), "-o", os.path.relpath(obj, ROOT)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")


def _link(objs, lib: str):
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", os.path.relpath(lib, ROOT)] + \
          [os.path.relpath(o, ROOT) for o in objs]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")


def verify(jobs: int = 0, keep: bool = False) -> dict:
    """Cold-build every csrc/*.hip into a fresh scratch directory (no stamps, no cached objects) and compare each
    object and the linked library with the shipped ``_hip/`` files byte for byte.  Proves that the library a run
    loads is exactly what these sources compile to on this machine's compiler."""
    import shutil
    import tempfile
    import time
    t0 = time.time()
    tmp = tempfile.mkdtemp(prefix="pathnet_cold_")
    try:
        srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
        objs = [os.path.join(tmp, os.path.basename(s) + ".o") for s in srcs]
        with cf.ThreadPoolExecutor(_jobs(jobs)) as ex:
            list(ex.map(lambda so: _compile(*so), zip(srcs, objs)))
        lib = os.path.join(tmp, os.path.basename(LIB))
        _link(objs, lib)
        per = {}
        for o in objs:
            shipped = os.path.join(OUT_DIR, os.path.basename(o))
            per[os.path.basename(o)] = os.path.exists(shipped) and _file_sha(shipped) == _file_sha(o)
        cold = _file_sha(lib)
        shipped = _file_sha(LIB) if os.path.exists(LIB) else ""
        return {"compiled_here": [os.path.basename(o) for o in objs], "sources_sha256": source_digest()[:16],
                "cold_lib_sha256": cold[:16], "shipped_lib_sha256": shipped[:16], "lib_equal": cold == shipped,
                "objects_equal": all(per.values()), "objects_differing": [k for k, v in per.items() if not v],
                "seconds": round(time.time() - t0, 1), "compiler": HIPCC, "arch": ARCH}
    finally:
        if not keep:
            shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    if "--verify" in sys.argv:
        import json
        j = int(sys.argv[sys.argv.index("--jobs") + 1]) if "--jobs" in sys.argv else 0
        print(json.dumps(verify(jobs=j)), flush=True)
    else:
        print(build(verbose="-v" in sys.argv))
