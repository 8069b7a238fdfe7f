"""ctypes binding to ``_native/libmls_kernels.so`` (the C ABI of ``csrc/*.hip``).

The library links ``libamdhip64.so.7``; torch-ROCm has already loaded its own copy with the
same soname, so the loader reuses it and our launches share torch's HIP runtime, streams and
graph capture (never load a second HIP runtime).  ``import torch`` therefore
happens before the ``CDLL``.

There is deliberately no silent fallback: if the library is missing on a machine that has a
GPU, :func:`lib` raises.  Callers that want the stock-PyTorch path ask for it explicitly
(``BACKEND=eager``).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch  # noqa: F401  (must load the HIP runtime first)

from . import build as _build

_c = ctypes
_LOCK = threading.Lock()
_LIB: Optional[ctypes.CDLL] = None

P = _c.c_void_p
I = _c.c_int
L = _c.c_long
F = _c.c_float
SZ = _c.c_size_t
FP = _c.POINTER(_c.c_float)

_SIGS = {
    "mls_conv2d": [P, P, P, P, P, P, P, SZ, I, I, I, I, I, I, I, I, I, I, I, I, P],
    "mls_conv2d_dual": [P, P, P, P, P, P, SZ, I, I, I, I, I, I, I, I, I, I, I, I, P],
    "mls_conv_chain": [P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, P],
    "mls_gemm": [P, P, P, P, P, P, P, SZ, I, I, I, I, I, I, P],
    "mls_gemm_heuristic": [I, I, I, _c.POINTER(I), _c.POINTER(I)],
    "mls_gemm_tile": [P, P, P, P, P, I, I, I, I, I, I, I, I, I, P, _c.c_longlong, P, I, P],
    "mls_gemm_tile_pick": [I, I],
    "mls_gemm_tile_ln": [P, P, P, P, P, I, I, I, I, I, P, P, P, P, _c.c_longlong, F, P],
    "mls_gemm_num_cfgs": [],
    "mls_normalize_u8": [P, P, I, I, I, I, FP, FP, P],
    "mls_maxpool2d": [P, P, I, I, I, I, I, I, I, P],
    "mls_stem_pool": [P, P, P, P, I, I, I, FP, FP, P],
    "mls_stem_pool_conv1": [P, P, P, P, I, I, I, FP, FP, P, P, P, P],
    "mls_conv3x3_halo": [P, P, P, P, P, P, SZ, I, I, I, I, I, I, I, I, P],
    "mls_conv3x3_halo_geometry": [I, I, I, _c.POINTER(I), _c.POINTER(I)],
    "mls_conv3x3_halo_geometry_v": [I, I, I, I, _c.POINTER(I), _c.POINTER(I)],
    "mls_conv2d_pool": [P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P],
    "mls_fc_head": [P, P, P, P, P, P, P, I, I, I, I, I, P, _c.c_longlong, P],
    "mls_conv3x3_pipe": [P, P, P, P, P, SZ, I, I, I, I, I, I, I, I, I, P],
    "mls_conv3x3_pipe_geometry": [I, I, I, I, _c.POINTER(I), _c.POINTER(I)],
    "mls_conv3x3_pipe_num_variants": [],
    "mls_avgpool_global": [P, P, I, I, I, P],
    "mls_bn_act": [P, P, P, P, L, I, I, P],
    "mls_silu_mul_interleaved": [P, P, L, I, P],
    "mls_softmax_topk": [P, I, P, P, I, I, I, I, F, P],
    "mls_softmax_rows": [P, P, P, I, I, I, F, P],
    "mls_topk_merge": [P, P, P, P, I, I, I, I, I, I, P],
    "mls_topk_chunks": [P, P, P, I, I, I, I, I, P],
    "mls_layernorm": [P, P, P, P, P, P, L, I, F, I, P],
    "mls_embed_ln": [P, P, P, P, P, P, P, P, L, I, I, I, F, P],
    "mls_embed_ln2": [P, P, I, P, P, P, P, P, P, P, P, L, I, I, I, F, P],
    "mls_embedding": [P, P, P, L, I, I, I, P],
    "mls_prefill_slots": [P, P, P, P, I, I, I, I, I, P, P],
    "mls_last_rows": [P, P, P, I, I, I, P, P, P],
    "mls_rope": [P, P, P, P, L, I, I, I, P],
    "mls_ar_create": [I, I, L, P],
    "mls_ar_create2": [I, I, L, L, P],
    "mls_ar_allreduce2": [P, P, P, L, _c.c_longlong, P],
    "mls_ar_handle": [P, P],
    "mls_ar_handle_size": [],
    "mls_ar_open": [P, P],
    "mls_ar_allreduce": [P, P, P, L, _c.c_longlong, P],
    "mls_ar_error": [P, P],
    "mls_ar_error_peek": [P, P, P],
    "mls_ar_set_timeout": [P, _c.c_longlong],
    "mls_ar_allgather": [P, P, P, L, _c.c_longlong, P],
    "mls_ar_reset": [P],
    "mls_gpu_sleep": [L, P],
    "mls_h2d_pull": [P, P, _c.c_longlong, I, P],
    "mls_h2d_pull_cell": [P, P, _c.c_longlong, I, P],
    "mls_d2h_push": [P, P, _c.c_longlong, I, P],
    "mls_stem_set_stamps": [P],
    "mls_stem_set_version": [I],
    "mls_flash_set_version": [I],
    "mls_image_decode": [P, P, P, L, I, P, P],
    "mls_decode_pick": [P, P, I, I, I, P, P, P, P, P, P, P, I, P, P, P, P, P],
    "mls_ar_destroy": [P],
    "mls_rope_kv": [P, P, P, P, L, I, I, I, I, P, P, P, P, I, I, L, I, I, P],
    "mls_kv_append": [P, I, I, I, P, P, P, L, I, I, I, P],
    "mls_flash_attention": [P, P, P, P, I, I, I, I, I, I, I, I, I, P, I, F, P],
    "mls_flash_attention_rows": [P, P, P, P, I, I, I, I, I, I, I, I, I, I, P, I, F, P],
    "mls_skinny_gemm": [P, P, P, P, P, P, SZ, I, I, I, I, I, P],
    "mls_mgemm": [P, P, P, P, P, P, SZ, I, I, I, I, I, I, P], "mls_mgemm_auto_split": [I, I, I],
    "mls_gemm_slabs": [P, P, P, SZ, I, I, I, I, I, P, P], "mls_splitk_add_rmsnorm": [P, SZ, I, I, I, P, P, P, F, P],
    "mls_skinny_gemm_norm": [P, P, P, P, P, P, P, P, SZ, I, I, I, I, I, I, F, P],
    "mls_skinny_pack": [P, P, I, I, P],
    "mls_skinny_packed": [P, P, P, P, P, P, P, I, I, I, I, I, F, I, P],
    "mls_decode_attention": [P, P, P, P, P, P, P, I, I, L, P, P, P, P, I, I, I, I, I, I, I, F, P, I, I, I, I, P],
    "mls_skinny_packed_combine": [P, P, P, P, I, I, I, I, P, P, P, P, I, I, I, I, I, P],
    "mls_skinny_packed_ar": [P, P, P, P, P, I, I, I, I, F, I, P, P],
    "mls_skinny_packed_combine_ar": [P, P, P, P, I, I, I, I, P, P, I, I, I, I, P, P],
    "mls_skinny_fp8": [P, P, P, P, P, P, P, P, I, I, I, I, I, F, I, P],
    "mls_stream_create_cumask": [P, I, _c.POINTER(P)],
    "mls_stream_get_cumask": [P, P, I],
    "mls_stream_destroy": [P],
    "mls_cu_census": [P, I, I, P],
}
_OPTIONAL_SIGS: dict = {"mls_set_debug_flags": [I], "mls_chain_set_l2_cw": [I],
    "mls_chain_set_l2_bm": [I],
    "mls_engine_launch": [P, P, P, _c.c_longlong, P, I, P, P, P, P, P], "mls_engine_launch_after": [P, P, P, P, _c.c_longlong, P, I, P, P, P, P, P], "mls_skinny_set_variant": [I], "mls_skinny_set_max_split": [I]}


class NativeError(RuntimeError):
    pass


def register_signatures(sigs: dict, optional: bool = False) -> None:
    """Extension point for kernel modules added later (attention, norms, collectives...)."""
    (_OPTIONAL_SIGS if optional else _SIGS).update(sigs)
    if _LIB is not None:
        _bind(_LIB)


def _bind(lib: ctypes.CDLL) -> None:
    for name, argtypes in list(_SIGS.items()) + list(_OPTIONAL_SIGS.items()):
        fn = getattr(lib, name, None)
        if fn is None:
            if name in _SIGS:
                raise NativeError(f"{name} missing from {lib._name}; rebuild the kernels")
            continue
        fn.argtypes = argtypes
        fn.restype = _c.c_int


DEBUG = os.environ.get("MLS_DEBUG", "0") == "1"
DEBUG_TUS = ("attention", "norm_ops", "stem_pool", "conv3x3_halo")  # translation units with MLS_CHECK bounds
DEBUG_CODES = {
    101: "rope/KV append: cache slot beyond the cache",
    102: "rope/KV append: position beyond the RoPE table",
    201: "decode attention: lens[b] exceeds the split grid (host context bound max_len too small)",
    202: "decode attention (rope mode): position outside the RoPE table or != lens - 1",
    301: "flash attention: kv_lens[b] > S",
}


def lib(build_if_missing: bool = True) -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        path = _build.lib_path(DEBUG)
        override = os.environ.get("MLS_LIB_OVERRIDE")  # A/B runs only: an alternative build of the same sources
        if override:
            build_if_missing = False
            path = override
        if build_if_missing:
            # incremental: a no-op when the stamp matches the sources
            try:
                path = _build.build(debug=DEBUG)
            except Exception as e:  # toolchain missing -> only OK if the .so already exists
                if not os.path.exists(path):
                    raise NativeError(f"native kernels unavailable and build failed: {e}") from e
        if not os.path.exists(path):
            raise NativeError(f"native kernel library not built: {path}")
        handle = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        _bind(handle)
        _LIB = handle
        return _LIB


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise NativeError(f"{what} failed with status {rc}")
    if DEBUG and not torch.cuda.is_current_stream_capturing():
        debug_check(what)


def debug_check(what: str = "kernel") -> None:
    """Debug builds: synchronise, then raise on the first bound a kernel recorded (and clear it)."""
    if not DEBUG:
        return
    torch.cuda.synchronize()
    buf = (_c.c_int * 4)()
    for tu in DEBUG_TUS:
        fn = getattr(lib(), f"mls_debug_read_{tu}", None)
        if fn is None:
            raise NativeError(f"{lib()._name} is not a debug build")
        fn.argtypes = [_c.c_void_p]
        fn.restype = _c.c_int
        if fn(_c.cast(buf, _c.c_void_p)) != 0:
            raise NativeError("mls_debug_read failed")
        if buf[0]:
            raise NativeError(f"{what}: bound violated [{buf[0]}] {DEBUG_CODES.get(buf[0], '?')} "
                              f"(block {buf[1]},{buf[2]} thread {buf[3]})")


def stream_ptr(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
