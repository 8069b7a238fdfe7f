"""Build the native front end in-tree (host C++, no GPU code).

``python -m mlmicroservicetemplate_amd.frontend.build`` compiles

* ``csrc/httpfront.cpp`` -> ``_native/_httpfront<EXT_SUFFIX>`` (pybind11 extension: epoll HTTP/1.1
  server + C++ dynamic batcher, see :mod:`.native`), and
* ``csrc/loadgen.cpp``   -> ``_native/mls_loadgen`` (closed-loop keep-alive HTTP load generator),
* ``../engine/csrc/staging.cpp`` -> ``engine/_native/_staging<EXT_SUFFIX>`` (the engine's host
  staging copy pool, :mod:`mlmicroservicetemplate_amd.engine.staging`).

In-tree like the kernel library (``ops/build.py``), so the artefacts travel with the repo
snapshot; rebuilt only when a source or the flags change (hash stamp).
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_native")
ENGINE_CSRC = os.path.join(os.path.dirname(HERE), "engine", "csrc")
ENGINE_OUT = os.path.join(os.path.dirname(HERE), "engine", "_native")
CXXFLAGS = ["-O2", "-std=c++17", "-Wall", "-Wno-unused-result", "-pthread"]


def ext_path() -> str:
    return os.path.join(OUT_DIR, "_httpfront" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def staging_path() -> str:
    return os.path.join(ENGINE_OUT, "_staging" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def loadgen_path() -> str:
    return os.path.join(OUT_DIR, "mls_loadgen")


def _cxx() -> str:
    for cand in (os.environ.get("CXX"), shutil.which("g++"), shutil.which("c++"), "/opt/rocm/llvm/bin/clang++"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("no C++ compiler found (g++ / clang++)")


def _stamp(src: str, flags, deps=()) -> str:
    h = hashlib.sha256(" ".join(flags).encode())
    for path in (src, *deps):
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _build_one(src: str, out: str, flags, verbose: bool, force: bool, deps=()) -> str:
    stamp = _stamp(src, flags, deps)
    sf = out + ".stamp"
    if not force and os.path.exists(out) and os.path.exists(sf):
        with open(sf) as f:
            if f.read().strip() == stamp:
                return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [_cxx(), *flags, src, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed for {src}:\n{r.stderr[-8000:]}")
    os.replace(out + ".tmp", out)
    with open(sf, "w") as f:
        f.write(stamp)
    return out


def build(force: bool = False, verbose: bool = False):
    import pybind11

    ext_flags = CXXFLAGS + ["-shared", "-fPIC", "-fvisibility=hidden", "-I", pybind11.get_include(),
                            "-I", sysconfig.get_paths()["include"]]
    ext = _build_one(os.path.join(CSRC, "httpfront.cpp"), ext_path(), ext_flags, verbose, force)
    lg = _build_one(os.path.join(CSRC, "loadgen.cpp"), loadgen_path(), CXXFLAGS, verbose, force)
    stg = _build_one(os.path.join(ENGINE_CSRC, "staging.cpp"), staging_path(), ext_flags + ["-O3"], verbose, force,
                     deps=(os.path.join(ENGINE_CSRC, "staging_core.h"),))
    return ext, lg, stg


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    args = ap.parse_args(argv)
    for p in build(force=args.force, verbose=args.verbose):
        print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
