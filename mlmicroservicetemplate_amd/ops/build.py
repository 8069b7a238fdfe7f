"""Build the in-tree native kernel library for gfx950.

``python -m mlmicroservicetemplate_amd.ops.build`` compiles every ``csrc/*.hip`` with
``hipcc --offload-arch=gfx950`` (cross-compiles without a GPU) into
``ops/_native/libmls_kernels.so`` -- in-tree, so the library travels with the repo snapshot to
the GPU box and is what the Python bindings load.  No hipify, no torch headers: the kernels
are plain HIP with a C ABI (``extern "C"`` launchers taking raw pointers + a hipStream_t), and
the Python side hands over tensor pointers and torch's current stream (so launches land in
the same stream -- and the same hipGraph capture -- as the surrounding PyTorch work).

Rebuilds are incremental: each object is keyed by a hash of its source, the shared headers and
the compiler flags.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from typing import List, Optional

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_native")
LIB_NAME = "libmls_kernels.so"
DEBUG_LIB_NAME = "libmls_kernels_debug.so"  # -DMLS_DEBUG: bounds-checked variant (MLS_DEBUG=1)
ARCH = os.environ.get("MLS_OFFLOAD_ARCH", "gfx950")
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]
if os.environ.get("MLS_GELU_ERF", "0") == "1":  # exact erf GELU in every GEMM epilogue (common.h gelu_fast)
    CXXFLAGS.append("-DMLS_GELU_ERF")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the kernels)")


def sources() -> List[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def headers() -> List[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hpp")))


def _digest(paths: List[str], extra: str = "") -> str:
    h = hashlib.sha256(extra.encode())
    for p in paths:
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()[:16]


def lib_path(debug: bool = False) -> str:
    return os.path.join(OUT_DIR, DEBUG_LIB_NAME if debug else LIB_NAME)


def _flags(debug: bool) -> List[str]:
    return CXXFLAGS + (["-DMLS_DEBUG"] if debug else [])


def _compile(src: str, hdr_hash: str, obj_dir: str, verbose: bool, debug: bool = False) -> str:
    flags = _flags(debug)
    key = _digest([src], hdr_hash + " ".join(flags))
    obj = os.path.join(obj_dir, os.path.basename(src).replace(".hip", f".{key}.o"))
    if os.path.exists(obj):
        return obj
    cmd = [hipcc(), *flags, "-I", CSRC, "-c", src, "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-8000:]}")
    os.replace(obj + ".tmp", obj)
    return obj


def _check_no_missing_stubs(so: str) -> None:
    """A kernel template whose host-side stub failed to instantiate links into a .so that only fails
    at dlopen ("undefined symbol: ...__device_stub__..."): refuse to install such a library."""
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    r = subprocess.run([nm, "-D", "--undefined-only", so], capture_output=True, text=True)
    missing = [ln.split()[-1] for ln in r.stdout.splitlines() if "__device_stub__" in ln]
    if missing:
        os.remove(so)
        raise RuntimeError(f"{os.path.basename(so)}: kernel stubs not instantiated: {missing[:4]}")


def build(force: bool = False, verbose: bool = False, jobs: Optional[int] = None, debug: bool = False) -> str:
    os.makedirs(OUT_DIR, exist_ok=True)
    obj_dir = os.path.join(OUT_DIR, "obj_debug" if debug else "obj")
    os.makedirs(obj_dir, exist_ok=True)
    srcs = sources()
    hdr_hash = _digest(headers())
    stamp = _digest(srcs + headers(), " ".join(_flags(debug)))
    out = lib_path(debug)
    stamp_file = out + ".stamp"
    if not force and os.path.exists(out) and os.path.exists(stamp_file):
        with open(stamp_file) as f:
            if f.read().strip() == stamp:
                return out
    jobs = jobs or min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr_hash, obj_dir, verbose, debug), srcs))
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-8000:]}")
    _check_no_missing_stubs(out + ".tmp")
    os.replace(out + ".tmp", out)
    with open(stamp_file, "w") as f:
        f.write(stamp)
    # drop stale objects
    live = set(objs)
    for f in os.listdir(obj_dir):
        p = os.path.join(obj_dir, f)
        if p not in live:
            try:
                os.remove(p)
            except OSError:
                pass
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--debug", action="store_true", help="the bounds-checked -DMLS_DEBUG variant")
    args = ap.parse_args(argv)
    path = build(force=args.force, verbose=args.verbose, debug=args.debug)
    print(path)
    return 0


if __name__ == "__main__":
    sys.exit(main())
