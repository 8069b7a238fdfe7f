"""Tensor-level wrappers over the hand-written CDNA4 kernels (T5).

Every op here runs the native HIP kernel on torch's current stream -- there is no eager
fallback for CUDA tensors (a missing library raises :class:`NativeError`).  The plain-PyTorch
oracles the kernels are tested against live in ``ops.reference``.

Layouts: activations NHWC / row-major ``[rows][features]`` bf16; conv weights
``[Cout][KH][KW][Cin]`` bf16 (see :func:`pack_conv_weight`); per-channel scale / bias fp32.
"""
from __future__ import annotations

from . import _lib  # noqa: F401  (re-exported: ops._lib.DEBUG, register_signatures)
from ._lib import NativeError, available, check, lib, stream_ptr  # noqa: F401
from ._core import (  # noqa: F401
    ACT_GELU,
    ACT_NONE,
    ACT_RELU,
    ACT_SILU,
    ACT_SILU_MUL,
    ACT_TANH,
    StreamWorkspace,
    conv_out_hw,
)
from .tables import (  # noqa: F401
    gemm_plan,
    gemm_tile_plan,
    load_blas_tuning,
    small_m_plan_for,
    tile_cfg_for,
    tile_route_for,
)
from .gemm_ops import (  # noqa: F401
    FP8_MAX,
    GEMM_TILE_CFGS,
    SPLIT_COUNTER_ELEMS,
    fold_layernorm,
    fold_norm,
    fp8_reference,
    gemm,
    gemm_heuristic,
    gemm_rmsnorm,
    gemm_tile,
    gemm_tile_ln,
    layernorm_from_partials,
    ln_partials,
    interleave_gate_up,
    pack_skinny,
    pack_skinny_fp8,
    pack_skinny_reference,
    silu_mul_interleaved,
    skinny_fp8,
    mgemm,
    skinny_packed,
    skinny_packed_ar,
    split_counters,
)
from .dispatch import (  # noqa: F401
    BLAS_MIN_M,
    TILE_MIN_M,
    mgemm_route,
    linear_add_rmsnorm,
    linear,
    linear_ln,
    ln_foldable,
)
from .softmax import (  # noqa: F401
    softmax_rows,
    softmax_topk,
    topk_large,
)
from .vision import (  # noqa: F401
    CFG_HALO,
    CFG_HALO_N32,
    CFG_HALO_XL,
    CFG_PIPE,
    CHAIN_SHAPES,
    HALO_CFGS,
    PIPE_CFGS,
    PIPE_VARIANTS,
    avgpool_global_nhwc,
    bn_act,
    conv1x1_chain,
    conv1x1_dual,
    conv2d_nhwc,
    conv2d_pool,
    conv3x3_halo,
    conv3x3_halo_geometry,
    conv3x3_pipe,
    conv3x3_pipe_geometry,
    fc_head,
    maxpool2d_nhwc,
    normalize_u8,
    pack_conv_weight,
    set_chain_l2_cw,
    stem_pool_u8,
)
from .transformer import (  # noqa: F401
    DecodePartials,
    decode_attention,
    decode_pick,
    embed_layernorm,
    embed_layernorm_packed,
    embedding,
    flash_attention,
    flash_attention_rows,
    kv_append,
    last_rows,
    layernorm,
    prefill_slots,
    rmsnorm,
    rope_,
    rope_kv_,
    skinny_packed_combine,
    skinny_packed_combine_ar,
)
from .image import (  # noqa: F401
    IMAGE_CONTAINER_BYTES,
    IMAGE_SCRATCH_PER_IMAGE,
    d2h_push,
    gpu_sleep,
    h2d_pull,
    h2d_pull_cell,
    image_decode,
)
from .partition import (  # noqa: F401
    MASK_WORDS,
    census_cus,
    cu_census,
    cu_masked_stream,
    intra_partition_words,
    partition_masks,
    xcd_cu_masks,
)

__all__ = [
    "NativeError",
    "available",
    "lib",
    "conv2d_nhwc",
    "gemm",
    "normalize_u8",
    "maxpool2d_nhwc",
    "avgpool_global_nhwc",
    "bn_act",
    "softmax_topk",
    "softmax_rows",
    "pack_conv_weight",
    "conv_out_hw",
    "gemm_heuristic",
]
