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


def _current(src: str, out: str, flags, deps=()) -> bool:
    sf = out + ".stamp"
    if not (os.path.exists(out) and os.path.exists(sf)):
        return False
    with open(sf) as f:
        return f.read().strip() == _stamp(src, flags, deps)


def _build_one(src: str, out: str, flags, verbose: bool, force: bool, deps=()) -> str:
    """Compile under an exclusive lock on ``<out>.lock`` into a per-process temp name, then an
    atomic rename: concurrent builders (several ranks starting together) never load or install a
    half-written module."""
    import fcntl

    if not force and _current(src, out, flags, deps):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and _current(src, out, flags, deps):  # another process built it meanwhile
            return out
        tmp = f"{out}.{os.getpid()}.tmp"
        cmd = [_cxx(), *flags, src, "-o", tmp]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            if os.path.exists(tmp):
                os.unlink(tmp)
            raise RuntimeError(f"build failed for {src}:\n{r.stderr[-8000:]}")
        os.replace(tmp, out)
        with open(out + ".stamp", "w") as f:
            f.write(_stamp(src, flags, deps))
    return out


def _ext_flags():
    import pybind11

    return CXXFLAGS + ["-shared", "-fPIC", "-fvisibility=hidden", "-I", pybind11.get_include(),
                       "-I", sysconfig.get_paths()["include"]]


def staging_current() -> bool:
    """Is the built staging module up to date with ``staging.cpp`` / ``staging_core.h``?"""
    return _current(os.path.join(ENGINE_CSRC, "staging.cpp"), staging_path(), _ext_flags() + ["-O3"],
                    (os.path.join(ENGINE_CSRC, "staging_core.h"),))


def build(force: bool = False, verbose: bool = False):
    ext_flags = _ext_flags()
    ext = _build_one(os.path.join(CSRC, "httpfront.cpp"), ext_path(), ext_flags, verbose, force,
                     deps=(os.path.join(CSRC, "jpeg_coefs.h"),))
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
