"""ResNet-path ops: implicit-GEMM / halo / pipelined convolutions with fused epilogues, the fused stem, pools, the fused classifier head."""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from ._lib import check, lib, stream_ptr
from ._core import ACT_NONE, ACT_RELU, _act, _need, _ptr, _workspace_args, conv_out_hw


def pack_conv_weight(w_oihw: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    """OIHW (PyTorch) -> ``[Cout][KH][KW][Cin]``.  Cin == 3 (image stem) is padded to 4 and KW to
    8 so one 16-byte chunk of the K dimension is two 4-channel taps (the kernel's stem mode)."""
    co, ci, kh, kw = w_oihw.shape
    w = w_oihw.permute(0, 2, 3, 1)
    if ci == 3 and kh > 1:
        w = torch.nn.functional.pad(w, (0, 1, 0, 8 - kw))  # Cin 3->4, KW -> 8
    return w.contiguous().to(dtype)


# conv2d_nhwc ``cfg`` values that select the halo-tiled direct 3x3 kernel (csrc/conv3x3_halo.hip,
# variant 0 / 1) instead of an implicit-GEMM tile config; tuning-table values like any other.
CFG_HALO = 100


CFG_HALO_N32 = 101


CFG_HALO_XL = 102  # 512 output pixels x 64 channels per block, 4 x 4 MFMA tiles per wave


HALO_CFGS = (CFG_HALO, CFG_HALO_N32, CFG_HALO_XL)


# cfg values that select the pipelined halo kernel (csrc/conv3x3_pipe.hip): CFG_PIPE + variant;
# the tuning table's splitk carries the K split, MLS items per block ride in the upper digits of
# splitk (splitk = ks + 16 * (ipb - 1)).
CFG_PIPE = 110


PIPE_VARIANTS = 12


PIPE_CFGS = tuple(range(CFG_PIPE, CFG_PIPE + PIPE_VARIANTS))


def conv2d_nhwc(
    x: torch.Tensor,
    w: torch.Tensor,
    bias: Optional[torch.Tensor] = None,
    *,
    kernel: int,
    stride: int = 1,
    pad: int = 0,
    scale: Optional[torch.Tensor] = None,
    residual: Optional[torch.Tensor] = None,
    act=ACT_NONE,
    out: Optional[torch.Tensor] = None,
    workspace: Optional[torch.Tensor] = None,
    cfg: int = 0,
    splitk: int = 0,
) -> torch.Tensor:
    """``act(conv(x, w) * scale + bias (+ residual))`` with x NHWC bf16 and w packed
    ``[Cout][KH][KW][Cin]`` (stem: ``[Cout][KH][8][4]`` on a pre-padded 4-channel image, pad 0)."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(w, "w", torch.bfloat16, dev)
    B, H, W, C = x.shape
    cout = w.shape[0]
    kh = kw = kernel
    if C == 4 and kernel > 1:
        if tuple(w.shape) != (cout, kh, 8, 4):
            raise ValueError(f"stem weight must be [Cout,{kh},8,4], got {tuple(w.shape)}")
    elif tuple(w.shape) != (cout, kh, kw, C):
        raise ValueError(f"weight shape {tuple(w.shape)} != [{cout},{kh},{kw},{C}]")
    if cout % 8:
        raise ValueError("Cout must be a multiple of 8")
    ho, wo = conv_out_hw(H, W, kernel, stride, pad)
    if cfg in PIPE_CFGS:
        if kernel != 3 or stride != 1 or pad != 1 or scale is not None or residual is not None:
            raise ValueError("CFG_PIPE: 3x3 / stride 1 / pad 1 convolutions without a scale / residual only")
        ks, ipb = max(1, int(splitk)) % 16 or 1, max(1, int(splitk)) // 16 + 1
        return conv3x3_pipe(x, w, bias, act=act, out=out, variant=cfg - CFG_PIPE, splitk=ks, ipb=ipb,
                            workspace=workspace)
    if cfg in HALO_CFGS:
        if kernel != 3 or stride != 1 or pad != 1 or scale is not None:
            raise ValueError("CFG_HALO: 3x3 / stride 1 / pad 1 convolutions without a scale only")
        return conv3x3_halo(x, w, bias, act=act, residual=residual, out=out, variant=cfg - CFG_HALO,
                            splitk=splitk, workspace=workspace)
    for name, t in (("bias", bias), ("scale", scale)):
        if t is not None:
            _need(t, name, torch.float32, dev)
            if t.numel() != cout:
                raise ValueError(f"{name} must have {cout} elements")
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (B, ho, wo, cout):
            raise ValueError(f"residual shape {tuple(residual.shape)} != {(B, ho, wo, cout)}")
    if out is None:
        out = torch.empty(B, ho, wo, cout, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != (B, ho, wo, cout):
            raise ValueError("out has wrong shape")
    wsp, wsb = _workspace_args(workspace)
    rc = lib().mls_conv2d(
        x.data_ptr(), w.data_ptr(), _ptr(scale), _ptr(bias), _ptr(residual), out.data_ptr(), wsp, wsb,
        B, H, W, C, cout, kh, kw, stride, pad, _act(act), cfg, splitk, stream_ptr(dev),
    )
    check(rc, "mls_conv2d")
    return out


def conv1x1_dual(y: torch.Tensor, x: torch.Tensor, w_cat: torch.Tensor, bias: Optional[torch.Tensor] = None, *,
                 stride2: int = 1, act=ACT_NONE, out: Optional[torch.Tensor] = None,
                 workspace: Optional[torch.Tensor] = None, cfg: int = 0, splitk: int = 0) -> torch.Tensor:
    """``act(conv1x1(y, W_y) + conv1x1_stride2(x, W_x) + bias)`` as ONE GEMM over the concatenated
    reduction (``w_cat`` = ``[Cout][Cin_y + Cin_x]``): a ResNet bottleneck's last conv fused with its
    downsample projection, so the identity branch is never materialised."""
    dev = y.device
    _need(y, "y", torch.bfloat16, dev)
    _need(x, "x", torch.bfloat16, dev)
    _need(w_cat, "w_cat", torch.bfloat16, dev)
    B, Ho, Wo, C1 = y.shape
    B2, H2, W2, C2 = x.shape
    cout = w_cat.shape[0]
    if B2 != B or tuple(w_cat.shape) != (cout, C1 + C2) or conv_out_hw(H2, W2, 1, stride2, 0) != (Ho, Wo):
        raise ValueError("conv1x1_dual: inconsistent shapes")
    if C1 % 64 or C2 % 8 or cout % 8:
        raise ValueError("conv1x1_dual needs Cin_y % 64 == 0, Cin_x % 8 == 0, Cout % 8 == 0")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
    if out is None:
        out = torch.empty(B, Ho, Wo, cout, device=dev, dtype=torch.bfloat16)
    wsp, wsb = _workspace_args(workspace)
    rc = lib().mls_conv2d_dual(y.data_ptr(), x.data_ptr(), w_cat.data_ptr(), _ptr(bias), out.data_ptr(), wsp, wsb,
                               B, Ho, Wo, C1, H2, W2, C2, stride2, cout, _act(act), cfg, splitk, stream_ptr(dev))
    check(rc, "mls_conv2d_dual")
    return out


# (K of the conv3 GEMM, N1, N2) csrc/conv_chain.hip is instantiated for
CHAIN_SHAPES = ((64, 256, 64), (128, 256, 64), (64, 256, 128), (128, 512, 128), (128, 512, 256), (256, 1024, 256))


def set_chain_l2_cw(cw: int) -> None:
    """A/B: output-channel chunk width of the layer2 chain boundaries (64 default, or 32)."""
    lib().mls_chain_set_l2_cw(int(cw))


def conv1x1_chain(a1: torch.Tensor, w3: torch.Tensor, b3: Optional[torch.Tensor], w1: torch.Tensor,
                  b1: Optional[torch.Tensor], *, residual: Optional[torch.Tensor] = None,
                  a2: Optional[torch.Tensor] = None, stride2: int = 1,
                  y_out: Optional[torch.Tensor] = None, t1_out: Optional[torch.Tensor] = None):
    """One bottleneck boundary in one kernel (csrc/conv_chain.hip):
    ``y = relu(conv1x1([a1 | a2 at stride2], w3) + b3 (+ residual))`` and
    ``t1 = relu(conv1x1(y, w1) + b1)``; y never makes an HBM round trip.  Returns ``(y, t1)``.
    ``w3`` is ``[N1][Ka (+ Kb)]`` (the dual concatenation when ``a2`` is given; no residual then),
    ``w1`` ``[N2][N1]``.  Supported (Ka + Kb, N1, N2): CHAIN_SHAPES -- the ResNet-50 layer1,
    layer2 and layer3 boundaries."""
    dev = a1.device
    _need(a1, "a1", torch.bfloat16, dev)
    _need(w3, "w3", torch.bfloat16, dev)
    _need(w1, "w1", torch.bfloat16, dev)
    B, Ho, Wo, Ka = a1.shape
    N1, N2 = w3.shape[0], w1.shape[0]
    if a2 is not None:
        _need(a2, "a2", torch.bfloat16, dev)
        if residual is not None:
            raise ValueError("conv1x1_chain: the dual form has no residual")
        B2, H2, W2, Kb = a2.shape
        if B2 != B or conv_out_hw(H2, W2, 1, stride2, 0) != (Ho, Wo):
            raise ValueError("conv1x1_chain: a2 does not match a1's grid at stride2")
    else:
        H2 = W2 = Kb = 0
    if w3.reshape(N1, -1).shape[1] != Ka + Kb or w1.reshape(N2, -1).shape[1] != N1:
        raise ValueError("conv1x1_chain: weight shapes do not chain")
    if (Ka + Kb, N1, N2) not in CHAIN_SHAPES:
        raise ValueError(f"conv1x1_chain: unsupported shape (K {Ka + Kb}, N1 {N1}, N2 {N2})")
    for name, t, n in (("b3", b3, N1), ("b1", b1, N2)):
        if t is not None:
            _need(t, name, torch.float32, dev)
            if t.numel() != n:
                raise ValueError(f"{name} must have {n} elements")
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (B, Ho, Wo, N1):
            raise ValueError("residual shape mismatch")
    y = torch.empty(B, Ho, Wo, N1, device=dev, dtype=torch.bfloat16) if y_out is None else y_out
    t1 = torch.empty(B, Ho, Wo, N2, device=dev, dtype=torch.bfloat16) if t1_out is None else t1_out
    rc = lib().mls_conv_chain(a1.data_ptr(), _ptr(a2), w3.data_ptr(), _ptr(b3), _ptr(residual), y.data_ptr(),
                              w1.data_ptr(), _ptr(b1), t1.data_ptr(), B, Ho, Wo, Ka, H2, W2, Kb, stride2, N1, N2,
                              stream_ptr(dev))
    check(rc, "mls_conv_chain")
    return y, t1


_MEAN_STD_CACHE = {}


def normalize_u8(images: torch.Tensor, mean, std, pad: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """uint8 ``[B,H,W,3]`` -> bf16 ``[B,H+2p,W+2p,4]`` = ((x - mean) / std, 0) with a zero border
    of ``pad`` pixels (the stem conv is then launched with pad 0 on the pre-padded image)."""
    dev = images.device
    _need(images, "images", torch.uint8, dev)
    B, H, W, C = images.shape
    if C != 3:
        raise ValueError("expected 3-channel images")
    shape = (B, H + 2 * pad, W + 2 * pad, 4)
    if out is None:
        out = torch.empty(shape, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != shape:
            raise ValueError(f"out must be {shape}")
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    rc = lib().mls_normalize_u8(images.data_ptr(), out.data_ptr(), B, H, W, pad, m, s, stream_ptr(dev))
    check(rc, "mls_normalize_u8")
    return out


def stem_pool_u8(images: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, mean, std,
                 out: Optional[torch.Tensor] = None, conv1_w: Optional[torch.Tensor] = None,
                 conv1_b: Optional[torch.Tensor] = None):
    """ResNet input block in one kernel: uint8 ``[B,224,224,3]`` -> normalise -> 7x7/2 conv
    (packed ``[64,7,8,4]`` weights, BN folded) + bias -> ReLU -> 3x3/2 max pool -> bf16
    ``[B,56,56,64]`` (csrc/stem_pool.hip).  With ``conv1_w`` (``[64, 64]`` or ``[64,1,1,64]``, BN
    folded) / ``conv1_b`` the first bottleneck's 1x1 conv + ReLU runs on each pooled tile in the
    same kernel and ``(pooled, t1)`` is returned."""
    dev = images.device
    _need(images, "images", torch.uint8, dev)
    _need(w, "w", torch.bfloat16, dev)
    _need(bias, "bias", torch.float32, dev)
    B, H, W, C = images.shape
    if C != 3 or H != 224 or W != 224 or tuple(w.shape) != (64, 7, 8, 4) or bias.numel() != 64:
        raise ValueError("stem_pool_u8: 224x224x3 images, [64,7,8,4] weights, 64 biases")
    shape = (B, 56, 56, 64)
    if out is None:
        out = torch.empty(shape, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != shape:
            raise ValueError(f"out must be {shape}")
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    if conv1_w is None:
        check(lib().mls_stem_pool(images.data_ptr(), w.data_ptr(), bias.data_ptr(), out.data_ptr(), B, H, W, m, s,
                                  stream_ptr(dev)), "mls_stem_pool")
        return out
    _need(conv1_w, "conv1_w", torch.bfloat16, dev)
    if conv1_w.numel() != 64 * 64 or conv1_w.shape[0] != 64:
        raise ValueError("stem_pool_u8: conv1_w must be [64, 64] (Cout x Cin)")
    if conv1_b is not None:
        _need(conv1_b, "conv1_b", torch.float32, dev)
        if conv1_b.numel() != 64:
            raise ValueError("conv1_b must have 64 elements")
    t1 = torch.empty(shape, device=dev, dtype=torch.bfloat16)
    check(lib().mls_stem_pool_conv1(images.data_ptr(), w.data_ptr(), bias.data_ptr(), out.data_ptr(), B, H, W, m, s,
                                    conv1_w.data_ptr(), _ptr(conv1_b), t1.data_ptr(), stream_ptr(dev)),
          "mls_stem_pool_conv1")
    return out, t1


def conv3x3_halo(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, act=ACT_NONE,
                 residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                 variant: int = 0, splitk: int = 1, workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """3x3 / stride 1 / pad 1 NHWC conv on the halo-tiled direct kernel (csrc/conv3x3_halo.hip):
    x ``[B,H,W,Cin]`` bf16, w packed ``[N,3,3,Cin]`` bf16, bias fp32 ``[N]`` -> ``[B,H,W,N]``
    ``act(conv + bias (+ residual))``.  Cin % 32 == 0; ``variant`` 0 = 64 output channels x 8
    waves per block (N % 64 == 0), 1 = 32 x 4 (N % 32 == 0), 2 = the XL tile (512 output pixels
    x 64 channels, 8 waves of 4 x 4 MFMA tiles).  ``splitk`` > 1 splits the input
    channels over that many blocks per tile, reduced in the same launch through fp32 slabs in
    ``workspace`` (>= splitk * B*H*W * N floats; otherwise, or on an uneven split, one slice)."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(w, "w", torch.bfloat16, dev)
    B, H, W, C = x.shape
    N = w.shape[0]
    if tuple(w.shape) != (N, 3, 3, C) or C % 32 or N % (32 if variant == 1 else 64) or variant not in (0, 1, 2):
        raise ValueError("conv3x3_halo: w must be [N,3,3,Cin], Cin % 32 == 0, N % 64 (variant 1: 32) == 0")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
        if bias.numel() != N:
            raise ValueError("bias must have N elements")
    shape = (B, H, W, N)
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != shape:
            raise ValueError(f"residual must be {shape}")
    if out is None:
        out = torch.empty(shape, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != shape:
            raise ValueError(f"out must be {shape}")
    wsp, wsb = _workspace_args(workspace)
    check(lib().mls_conv3x3_halo(x.data_ptr(), w.data_ptr(), _ptr(bias), _ptr(residual), out.data_ptr(), wsp, wsb,
                                 B, H, W, C, N, _act(act), variant, max(1, int(splitk)), stream_ptr(dev)),
          "mls_conv3x3_halo")
    return out


def conv2d_pool(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], pool: torch.Tensor, *, kernel: int,
                stride: int = 1, pad: int = 0, residual: Optional[torch.Tensor] = None, act=ACT_NONE,
                out: Optional[torch.Tensor] = None, pool_only: bool = True, cfg: int = 0) -> Optional[torch.Tensor]:
    """``conv2d_nhwc`` with the global average pool of its output fused into the epilogue (the
    network's last convolution, csrc/conv_gemm.hip ``ConvArgs::pool``): ``pool`` fp32 ``[B, Cout]``
    += the per-image mean of ``act(conv + bias (+ residual))``.  ``pool`` must be zero on entry
    (:func:`fc_head` zeroes it after reading); with ``pool_only`` the output is not written."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(w, "w", torch.bfloat16, dev)
    _need(pool, "pool", torch.float32, dev)
    B, H, W, C = x.shape
    cout = w.shape[0]
    if tuple(w.shape) != (cout, kernel, kernel, C) or C == 4:
        raise ValueError(f"weight shape {tuple(w.shape)} != [{cout},{kernel},{kernel},{C}]")
    ho, wo = conv_out_hw(H, W, kernel, stride, pad)
    if pool.shape[0] < B or pool.shape[-1] != cout:
        raise ValueError(f"pool must be [>= {B}, {cout}]")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
    if residual is not None:
        _need(residual, "residual", torch.bfloat16, dev)
        if tuple(residual.shape) != (B, ho, wo, cout):
            raise ValueError("residual shape mismatch")
    if not pool_only and out is None:
        out = torch.empty(B, ho, wo, cout, device=dev, dtype=torch.bfloat16)
    check(lib().mls_conv2d_pool(x.data_ptr(), w.data_ptr(), None, _ptr(bias), _ptr(residual), _ptr(out),
                                pool.data_ptr(), int(pool_only), B, H, W, C, cout, kernel, kernel, stride, pad,
                                _act(act), int(cfg), stream_ptr(dev)), "mls_conv2d_pool")
    return out


def fc_head(pooled: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], k: int, *,
            logits: Optional[torch.Tensor] = None, softmax: bool = True, err: Optional[torch.Tensor] = None,
            vals: Optional[torch.Tensor] = None, idx: Optional[torch.Tensor] = None):
    """Classifier head in one launch (csrc/head.hip): ``pooled`` fp32 ``[B, K]`` (the fused average
    pool; ZEROED by this call for the next forward) -> logits = pooled . w^T + bias (fp32, into
    ``logits``) -> (softmax ->) top-``k``.  ``err`` int32 ``[B]``: rows flagged nonzero come back
    with ids -1 and NaN values (an undecodable upload).  Returns (vals fp32 [B,k], ids int32 [B,k],
    logits); with ``k == 0`` only the logits."""
    dev = pooled.device
    _need(pooled, "pooled", torch.float32, dev)
    _need(w, "w", torch.bfloat16, dev)
    B, K = pooled.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError("w must be [N, K]")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
    if logits is None:
        logits = torch.empty(B, N, device=dev, dtype=torch.float32)
    _need(logits, "logits", torch.float32, dev)
    if logits.numel() < B * N:
        raise ValueError("logits buffer too small")
    if err is not None:
        _need(err, "err", torch.int32, dev)
    if k > 0:
        if vals is None:
            vals = torch.empty(B, k, device=dev, dtype=torch.float32)
        if idx is None:
            idx = torch.empty(B, k, device=dev, dtype=torch.int32)
    # the v2 kernels' per-K-slice partial slabs come from the torch allocator (inside a capture:
    # the graph's own pool, alive as long as the graph), never from a buffer the library frees
    ws = torch.empty((K // 256) * B * N if K % 256 == 0 else 0, device=dev, dtype=torch.float32)
    check(lib().mls_fc_head(pooled.data_ptr(), w.data_ptr(), _ptr(bias), logits.data_ptr(), _ptr(vals), _ptr(idx),
                            _ptr(err), B, N, K, int(k), int(softmax), ws.data_ptr() if ws.numel() else None,
                            ws.numel() * 4, stream_ptr(dev)), "mls_fc_head")
    return vals, idx, logits


def conv3x3_pipe(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, act=ACT_NONE,
                 out: Optional[torch.Tensor] = None, variant: int = 0, splitk: int = 1, ipb: int = 1,
                 workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """3x3 / stride 1 / pad 1 NHWC conv on the pipelined halo kernel (csrc/conv3x3_pipe.hip):
    x ``[B,H,W,Cin]`` bf16, w packed ``[N,3,3,Cin]`` bf16, bias fp32 ``[N]`` -> ``[B,H,W,N]``
    ``act(conv + bias)`` (act: none / ReLU).  ``variant`` picks (channels per item, waves, row
    blocks per wave, ring stages); ``splitk`` > 1 splits the input channels over that many items
    per tile (in-launch reduction through fp32 slabs in ``workspace``, >= splitk * B*H*W*N floats;
    otherwise one slice); ``ipb`` = consecutive items per block."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(w, "w", torch.bfloat16, dev)
    B, H, W, C = x.shape
    N = w.shape[0]
    if tuple(w.shape) != (N, 3, 3, C) or C % 32 or N % 32 or N > 512 or not 0 <= variant < PIPE_VARIANTS:
        raise ValueError("conv3x3_pipe: w must be [N,3,3,Cin], Cin % 32 == 0, N % 32 == 0, N <= 512")
    if act not in (ACT_NONE, ACT_RELU, "none", "relu"):
        raise ValueError("conv3x3_pipe: act must be none or relu")
    if bias is not None:
        _need(bias, "bias", torch.float32, dev)
        if bias.numel() != N:
            raise ValueError("bias must have N elements")
    shape = (B, H, W, N)
    if out is None:
        out = torch.empty(shape, device=dev, dtype=torch.bfloat16)
    else:
        _need(out, "out", torch.bfloat16, dev)
        if tuple(out.shape) != shape:
            raise ValueError(f"out must be {shape}")
    wsp, wsb = _workspace_args(workspace)
    check(lib().mls_conv3x3_pipe(x.data_ptr(), w.data_ptr(), _ptr(bias), out.data_ptr(), wsp, wsb, B, H, W, C, N,
                                 _act(act), int(variant), max(1, int(splitk)), max(1, int(ipb)), stream_ptr(dev)),
          "mls_conv3x3_pipe")
    return out


def conv3x3_pipe_geometry(B: int, H: int, W: int, variant: int = 0) -> Optional[Tuple[int, int]]:
    """(output rows per item, images per item) of the pipelined kernel's variant, or None."""
    th, nb = ctypes.c_int(0), ctypes.c_int(0)
    rc = lib().mls_conv3x3_pipe_geometry(B, H, W, variant, ctypes.byref(th), ctypes.byref(nb))
    return (th.value, nb.value) if rc == 0 else None


def conv3x3_halo_geometry(B: int, H: int, W: int, variant: int = 0) -> Optional[Tuple[int, int]]:
    """(output rows per tile, images per tile) the halo kernel uses for this shape, or None."""
    th, nb = ctypes.c_int(0), ctypes.c_int(0)
    rc = lib().mls_conv3x3_halo_geometry_v(B, H, W, variant, ctypes.byref(th), ctypes.byref(nb))
    return (th.value, nb.value) if rc == 0 else None


def maxpool2d_nhwc(x: torch.Tensor, k: int = 3, s: int = 2, p: int = 1, out: Optional[torch.Tensor] = None):
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    B, H, W, C = x.shape
    ho, wo = conv_out_hw(H, W, k, s, p)
    if out is None:
        out = torch.empty(B, ho, wo, C, device=dev, dtype=torch.bfloat16)
    rc = lib().mls_maxpool2d(x.data_ptr(), out.data_ptr(), B, H, W, C, k, s, p, stream_ptr(dev))
    check(rc, "mls_maxpool2d")
    return out


def avgpool_global_nhwc(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    B, H, W, C = x.shape
    if out is None:
        out = torch.empty(B, C, device=dev, dtype=torch.bfloat16)
    rc = lib().mls_avgpool_global(x.data_ptr(), out.data_ptr(), B, H * W, C, stream_ptr(dev))
    check(rc, "mls_avgpool_global")
    return out


def bn_act(x: torch.Tensor, scale: torch.Tensor, bias: torch.Tensor, relu: bool = False, out=None) -> torch.Tensor:
    """Standalone inference BatchNorm over the last (channel) dim (K3 unfused path)."""
    dev = x.device
    _need(x, "x", torch.bfloat16, dev)
    _need(scale, "scale", torch.float32, dev)
    _need(bias, "bias", torch.float32, dev)
    C = x.shape[-1]
    out = torch.empty_like(x) if out is None else out
    rc = lib().mls_bn_act(x.data_ptr(), out.data_ptr(), scale.data_ptr(), bias.data_ptr(), x.numel() // C, C,
                          int(relu), stream_ptr(dev))
    check(rc, "mls_bn_act")
    return out
