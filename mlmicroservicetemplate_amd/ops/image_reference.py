"""NumPy specification of the GPU image-container decode (``ops/csrc/image_decode.hip``).

A container (``frontend/csrc/jpeg_coefs.h``) holds either a raw 224 x 224 x 3 RGB image or the
dequantised DCT coefficients of a baseline JPEG plus the resize / crop geometry of the PIL
reference pipeline (``plugins.builtin.decode_image``: draft, RGB, shorter side 256 by bilinear
resampling, centre crop 224).  This module computes what the kernels compute, step for step:

1. IDCT of each block's s x s coefficient corner (s = 8 / DCT downscale), + 128, round, clamp;
2. chroma upsampling as libjpeg(-turbo) does it: "fancy" triangle filters for 2:1 horizontal
   (h2v1) and 2:1 both ways (h2v2), edge samples replicated; plain replication otherwise;
3. YCbCr -> RGB with libjpeg's 16-bit fixed-point tables;
4. Pillow's BILINEAR resample (separable, horizontal pass first, each pass rounded to uint8, with
   Pillow's fixed-point (22 fractional bits) coefficients, support widened by the downscale factor)
   evaluated only on the centre-crop window.

Used by the CPU tests as the oracle for the kernels and, against PIL itself, to pin how close the
GPU path is to the reference decode (tests/test_image_decode.py).
"""
from __future__ import annotations

import math
import struct
from typing import Tuple

import numpy as np

HDR = 64
OUT = 224
PAYLOAD = OUT * OUT * 3
CONTAINER_BYTES = HDR + PAYLOAD
MAGIC = 0x4A534C4D


def parse_header(buf) -> dict:
    b = bytes(buf[:HDR])
    magic, kind, w, h, nc, s, hmax, vmax = struct.unpack_from("<IIHHBBBB", b, 0)
    if magic != MAGIC:
        raise ValueError("not an image container")
    comps = []
    for c in range(3):
        ch, cv, bw, bh, off = struct.unpack_from("<BBHHI", b, 16 + 10 * c)
        comps.append(dict(h=ch, v=cv, bw=bw, bh=bh, offset=off))
    rw, rh, left, top, coarser, nblocks, entries_off = struct.unpack_from("<HHHHBII", b, 46)
    return dict(kind=kind, width=w, height=h, ncomp=nc, s=s, hmax=hmax, vmax=vmax, comps=comps[:nc], rw=rw, rh=rh,
                left=left, top=top, coarser=coarser, nblocks=nblocks, entries_off=entries_off)


def idct_matrix(s: int) -> np.ndarray:
    """M[x][u] = C(u)/2 * cos((2x + 1) u pi / 2s): pixel block = M @ F @ M.T (+128)."""
    m = np.zeros((s, s))
    for x in range(s):
        for u in range(s):
            cu = math.sqrt(0.5) if u == 0 else 1.0
            m[x, u] = cu / 2.0 * math.cos((2 * x + 1) * u * math.pi / (2 * s))
    return m


def coefficients(buf, hdr) -> np.ndarray:
    """The compact entries back to dense DEQUANTISED blocks ``[nblocks, s*s]`` (float64): block b's
    units start at gstart[b // 64] + sum(counts[64 * (b // 64): b]); an int8 value times the
    component's quantisation step, or the (0x80, pos) escape followed by an int16 unit."""
    s, nb = hdr["s"], hdr["nblocks"]
    pay = np.frombuffer(bytes(buf[HDR:]), dtype=np.uint8)
    qtab = pay[:384].view(np.uint16).reshape(3, 64).astype(np.float64)
    groups = (nb + 63) // 64
    gstart = pay[384: 384 + 4 * groups].view(np.uint32).astype(np.int64)
    counts_off = 384 + 4 * groups
    counts = pay[counts_off: counts_off + nb].astype(np.int64)
    ent = pay[hdr["entries_off"]:]
    comp_of = np.zeros(nb, np.int64)
    for ci, c in enumerate(hdr["comps"]):
        comp_of[c["offset"]: c["offset"] + c["bw"] * c["bh"]] = ci
    dense = np.zeros((nb, s * s))
    for b in range(nb):
        g = b // 64
        u = int(gstart[g] + counts[64 * g: b].sum())
        end = u + int(counts[b])
        q = qtab[comp_of[b]]
        while u < end:
            v, pos = int(np.int8(ent[2 * u])), int(ent[2 * u + 1])
            if v == -128:
                v = int(np.frombuffer(ent[2 * u + 2: 2 * u + 4].tobytes(), np.int16)[0])
                u += 2
            else:
                u += 1
            dense[b, pos] = v * q[pos]
    return dense


def planes(buf, hdr) -> list:
    s = hdr["s"]
    m = idct_matrix(s)
    out = []
    dense = coefficients(buf, hdr)
    for c in hdr["comps"]:
        n = c["bw"] * c["bh"]
        co = dense[c["offset"]: c["offset"] + n].reshape(c["bh"], c["bw"], s, s)
        px = np.einsum("xu,abuv,yv->abxy", m, co, m)  # [bh, bw, s(y), s(x)]
        px = np.clip(np.floor(px + 128.0 + 0.5), 0, 255).astype(np.int32)
        out.append(px.transpose(0, 2, 1, 3).reshape(c["bh"] * s, c["bw"] * s))
    return out


def _fancy_h2v1(p: np.ndarray, wo: int) -> np.ndarray:
    n = p.shape[1]
    o = np.zeros((p.shape[0], 2 * n), np.int32)
    if n == 1:
        o[:, 0] = o[:, 1] = p[:, 0]
        return o[:, :wo]
    o[:, 0] = p[:, 0]
    o[:, 1] = (p[:, 0] * 3 + p[:, 1] + 2) >> 2
    c = np.arange(1, n - 1)
    o[:, 2 * c] = (p[:, c] * 3 + p[:, c - 1] + 1) >> 2
    o[:, 2 * c + 1] = (p[:, c] * 3 + p[:, c + 1] + 2) >> 2
    o[:, 2 * n - 2] = (p[:, n - 1] * 3 + p[:, n - 2] + 1) >> 2
    o[:, 2 * n - 1] = p[:, n - 1]
    return o[:, :wo]


def _fancy_h2v2(p: np.ndarray, wo: int, ho: int) -> np.ndarray:
    hh, n = p.shape
    up = np.vstack([p[:1], p[:-1]])  # row above (edge replicated)
    dn = np.vstack([p[1:], p[-1:]])  # row below
    o = np.zeros((2 * hh, 2 * n), np.int32)
    for half, nb in ((0, up), (1, dn)):
        t = p * 3 + nb  # this column's vertical sum
        r = o[half::2]
        if n == 1:
            r[:, 0] = (t[:, 0] * 4 + 8) >> 4
            r[:, 1] = (t[:, 0] * 4 + 7) >> 4
            continue
        r[:, 0] = (t[:, 0] * 4 + 8) >> 4
        r[:, 1] = (t[:, 0] * 3 + t[:, 1] + 7) >> 4
        c = np.arange(1, n - 1)
        r[:, 2 * c] = (t[:, c] * 3 + t[:, c - 1] + 8) >> 4
        r[:, 2 * c + 1] = (t[:, c] * 3 + t[:, c + 1] + 7) >> 4
        r[:, 2 * n - 2] = (t[:, n - 1] * 3 + t[:, n - 2] + 8) >> 4
        r[:, 2 * n - 1] = (t[:, n - 1] * 4 + 7) >> 4
    return o[:ho, :wo]


def upsampled_component(p: np.ndarray, c: dict, hdr: dict) -> np.ndarray:
    """Component plane -> full-resolution samples [height][width] (libjpeg's per-component rule)."""
    W, H, s = hdr["width"], hdr["height"], hdr["s"]
    fx, fy = hdr["hmax"] // c["h"], hdr["vmax"] // c["v"]
    # the component's real (non-padding) extent, as libjpeg's downsampled_width / height
    cw = -(-W * c["h"] // hdr["hmax"])
    chh = -(-H * c["v"] // hdr["vmax"])
    p = p[:chh, :cw]
    if fx == 1 and fy == 1:
        return p[:H, :W]
    if fx == 2 and fy == 1 and s > 1:
        return _fancy_h2v1(p, W)[:H]
    if fx == 2 and fy == 2 and s > 1:
        return _fancy_h2v2(p, W, H)
    return np.repeat(np.repeat(p, fy, axis=0), fx, axis=1)[:H, :W]


def ycc_to_rgb(y: np.ndarray, cb: np.ndarray, cr: np.ndarray) -> np.ndarray:
    one_half = 1 << 15

    def fix(x):
        return int(x * (1 << 16) + 0.5)

    x_cb, x_cr = cb.astype(np.int64) - 128, cr.astype(np.int64) - 128
    r = y + ((fix(1.40200) * x_cr + one_half) >> 16)
    g = y + ((-fix(0.34414) * x_cb - fix(0.71414) * x_cr + one_half) >> 16)
    b = y + ((fix(1.77200) * x_cb + one_half) >> 16)
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)


PRECISION_BITS = 32 - 8 - 2


def resample_coeffs(in_size: int, out_size: int) -> Tuple[np.ndarray, np.ndarray, int]:
    """Pillow's precompute_coeffs for the bilinear filter: (xmin, fixed-point kernels, ksize)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros(out_size, np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ww = 0.0
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        k = np.zeros(ksize)
        for x in range(xmax):
            t = (x + xmin - center + 0.5) * ss
            w = 1.0 - abs(t) if abs(t) < 1.0 else 0.0
            k[x] = w
            ww += w
        for x in range(xmax):
            if ww != 0.0:
                k[x] /= ww
        for x in range(ksize):
            v = k[x] * (1 << PRECISION_BITS)
            kk[xx, x] = int(v + 0.5) if v >= 0 else int(v - 0.5)
        bounds[xx] = xmin
    return bounds, kk, ksize


def _clip8(v):
    return np.clip(v >> PRECISION_BITS, 0, 255)


def resize_crop(rgb: np.ndarray, hdr: dict) -> np.ndarray:
    H, W = rgb.shape[:2]
    rw, rh, left, top = hdr["rw"], hdr["rh"], hdr["left"], hdr["top"]
    img = rgb.astype(np.int64)
    if (rw, rh) != (W, H):
        if rw != W:
            bx, kx, ks = resample_coeffs(W, rw)
            cols = np.arange(left, left + OUT)
            acc = np.full((H, OUT, 3), 1 << (PRECISION_BITS - 1), np.int64)
            for j in range(ks):
                idx = np.clip(bx[cols] + j, 0, W - 1)
                acc += img[:, idx, :] * kx[cols, j][None, :, None]
            img = _clip8(acc)
        else:
            img = img[:, left:left + OUT]
        if rh != H:
            by, ky, ks = resample_coeffs(H, rh)
            rows = np.arange(top, top + OUT)
            acc = np.full((OUT, OUT, 3), 1 << (PRECISION_BITS - 1), np.int64)
            for j in range(ks):
                idx = np.clip(by[rows] + j, 0, H - 1)
                acc += img[idx, :, :] * ky[rows, j][:, None, None]
            img = _clip8(acc)
        else:
            img = img[top:top + OUT]
        return img.astype(np.uint8)
    return rgb[top:top + OUT, left:left + OUT].astype(np.uint8)


def decode_container(buf) -> np.ndarray:
    """Container -> uint8 [224, 224, 3] exactly as the GPU kernels produce it."""
    hdr = parse_header(buf)
    if hdr["kind"] == 0:
        return np.frombuffer(bytes(buf[HDR:HDR + PAYLOAD]), np.uint8).reshape(OUT, OUT, 3).copy()
    ps = planes(buf, hdr)
    comps = [upsampled_component(p, c, hdr) for p, c in zip(ps, hdr["comps"])]
    if hdr["ncomp"] == 1:
        rgb = np.repeat(comps[0][..., None], 3, axis=-1).astype(np.uint8)
    else:
        rgb = ycc_to_rgb(comps[0].astype(np.int64), comps[1], comps[2])
    return resize_crop(rgb, hdr)
