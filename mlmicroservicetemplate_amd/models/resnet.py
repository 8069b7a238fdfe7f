"""ResNet-50 v1.5 (stride on the 3x3 conv) for MI355X serving.

Three execution paths over ONE parameter set:

* ``resnet50_reference``  -- plain fp32 PyTorch functional ops (NCHW).  This is the
  numerics oracle for the HIP kernels (SURVEY.md §4 "Models" row).
* ``ResNet50Eager``       -- stock PyTorch-ROCm ops (MIOpen conv / hipBLASLt GEMM) in
  bf16 channels-last.  This is the in-repo *comparison baseline (b)* of SURVEY.md §6:
  the reference itself publishes no numbers.
* ``ResNet50Fused``       -- our hand-written CDNA4 kernels (``ops``): implicit-GEMM
  MFMA convs with BN folded into the epilogue (+residual +ReLU), max/avg pool, FC,
  softmax and top-k, NHWC end-to-end, capturable into one hipGraph per batch bucket.

The reference "model" is a constant-returning stub (reference ``src/model/model.py:23-31``);
the GPU models here have no reference counterpart and come from BASELINE.json's configs.
Weights are random-init (no network for checkpoints): kaiming-normal convs, BN with
non-trivial random running statistics so that BN folding is actually exercised.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

# (blocks, mid channels, out channels, first stride) per stage
STAGES: Tuple[Tuple[int, int, int, int], ...] = (
    (3, 64, 256, 1),
    (4, 128, 512, 2),
    (6, 256, 1024, 2),
    (3, 512, 2048, 2),
)
IMAGENET_MEAN = (0.485 * 255, 0.456 * 255, 0.406 * 255)
IMAGENET_STD = (0.229 * 255, 0.224 * 255, 0.225 * 255)
NUM_CLASSES = 1000


@dataclass
class ConvSpec:
    name: str
    cin: int
    cout: int
    k: int
    stride: int
    pad: int


def conv_specs() -> List[ConvSpec]:
    """All 53 convolutions of ResNet-50 v1.5 in execution order."""
    specs = [ConvSpec("stem", 3, 64, 7, 2, 3)]
    cin = 64
    for si, (nblocks, mid, cout, stride) in enumerate(STAGES):
        for bi in range(nblocks):
            s = stride if bi == 0 else 1
            p = f"layer{si + 1}.{bi}"
            specs.append(ConvSpec(p + ".conv1", cin, mid, 1, 1, 0))
            specs.append(ConvSpec(p + ".conv2", mid, mid, 3, s, 1))
            specs.append(ConvSpec(p + ".conv3", mid, cout, 1, 1, 0))
            if bi == 0:
                specs.append(ConvSpec(p + ".down", cin, cout, 1, s, 0))
            cin = cout
    return specs


def init_resnet50(seed: int = 0, num_classes: int = NUM_CLASSES) -> Dict[str, torch.Tensor]:
    """Random-init fp32 parameters on CPU. Conv weights are OIHW (PyTorch layout)."""
    g = torch.Generator().manual_seed(seed)
    params: Dict[str, torch.Tensor] = {}
    for spec in conv_specs():
        fan_in = spec.cin * spec.k * spec.k
        w = torch.randn(spec.cout, spec.cin, spec.k, spec.k, generator=g) * math.sqrt(2.0 / fan_in)
        params[spec.name + ".w"] = w
        c = spec.cout
        # zero-ish gamma on the last BN of each block (as in "zero-init residual") would make
        # the residual branch vanish and hide kernel bugs, so use O(1) random values instead.
        params[spec.name + ".bn.gamma"] = 0.5 + 0.5 * torch.rand(c, generator=g)
        params[spec.name + ".bn.beta"] = 0.1 * torch.randn(c, generator=g)
        params[spec.name + ".bn.mean"] = 0.1 * torch.randn(c, generator=g)
        params[spec.name + ".bn.var"] = 0.5 + torch.rand(c, generator=g)
    params["fc.w"] = torch.randn(num_classes, 2048, generator=g) * math.sqrt(1.0 / 2048)
    params["fc.b"] = 0.01 * torch.randn(num_classes, generator=g)
    return params


_BN = {"weight": "gamma", "bias": "beta", "running_mean": "mean", "running_var": "var"}


def torchvision_name(k: str) -> Optional[str]:
    """torchvision ``resnet50().state_dict()`` key -> this model's name (None: not a parameter)."""
    if k.endswith("num_batches_tracked"):
        return None
    p = k.split(".")
    if p[0] == "conv1":
        return "stem.w"
    if p[0] == "bn1":
        return f"stem.bn.{_BN[p[1]]}"
    if p[0] == "fc":
        return {"weight": "fc.w", "bias": "fc.b"}[p[1]]
    if p[0].startswith("layer") and len(p) >= 4:
        blk = f"{p[0]}.{p[1]}"
        if p[2].startswith("conv"):
            return f"{blk}.{p[2]}.w"
        if p[2].startswith("bn"):
            return f"{blk}.conv{p[2][2:]}.bn.{_BN[p[3]]}"
        if p[2] == "downsample":
            return f"{blk}.down.w" if p[3] == "0" else f"{blk}.down.bn.{_BN[p[4]]}"
    return k


def load_resnet50(path: str, num_classes: int = NUM_CLASSES) -> Dict[str, torch.Tensor]:
    """fp32 parameters from a safetensors checkpoint in this model's names or torchvision's
    (validated name by name, shape by shape)."""
    from ..utils.checkpoint import load_validated

    spec = {k: (tuple(v.shape), torch.float32) for k, v in init_resnet50_spec(num_classes).items()}
    return load_validated(path, spec, rename=lambda k: k if k in spec else torchvision_name(k))


def init_resnet50_spec(num_classes: int = NUM_CLASSES) -> Dict[str, torch.Tensor]:
    """Meta tensors with the shapes/dtypes of :func:`init_resnet50` (what non-source ranks need
    to receive the X1 weight broadcast without generating weights themselves)."""
    out: Dict[str, torch.Tensor] = {}
    for spec in conv_specs():
        out[spec.name + ".w"] = torch.empty(spec.cout, spec.cin, spec.k, spec.k, device="meta")
        for n in ("gamma", "beta", "mean", "var"):
            out[f"{spec.name}.bn.{n}"] = torch.empty(spec.cout, device="meta")
    out["fc.w"] = torch.empty(num_classes, 2048, device="meta")
    out["fc.b"] = torch.empty(num_classes, device="meta")
    return out


BN_EPS = 1e-5


def fold_bn(params: Dict[str, torch.Tensor], name: str) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-output-channel (scale, bias) so that BN(conv(x)) == conv(x) * scale + bias."""
    gamma = params[name + ".bn.gamma"]
    beta = params[name + ".bn.beta"]
    mean = params[name + ".bn.mean"]
    var = params[name + ".bn.var"]
    scale = gamma / torch.sqrt(var + BN_EPS)
    bias = beta - mean * scale
    return scale, bias


def normalize_reference(images_u8_nhwc: torch.Tensor) -> torch.Tensor:
    """uint8 NHWC -> fp32 NCHW normalised with ImageNet mean/std."""
    x = images_u8_nhwc.float()
    mean = torch.tensor(IMAGENET_MEAN, device=x.device)
    std = torch.tensor(IMAGENET_STD, device=x.device)
    x = (x - mean) / std
    return x.permute(0, 3, 1, 2).contiguous()


def _ref_conv_bn(params, x, spec: ConvSpec, relu: bool, residual=None):
    y = F.conv2d(x, params[spec.name + ".w"], stride=spec.stride, padding=spec.pad)
    y = F.batch_norm(
        y,
        params[spec.name + ".bn.mean"],
        params[spec.name + ".bn.var"],
        params[spec.name + ".bn.gamma"],
        params[spec.name + ".bn.beta"],
        training=False,
        eps=BN_EPS,
    )
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


def resnet50_reference(params: Dict[str, torch.Tensor], images_u8_nhwc: torch.Tensor) -> torch.Tensor:
    """fp32 logits [B, num_classes]; the oracle for every other path."""
    specs = {s.name: s for s in conv_specs()}
    x = normalize_reference(images_u8_nhwc)
    x = _ref_conv_bn(params, x, specs["stem"], relu=True)
    x = F.max_pool2d(x, kernel_size=3, stride=2, padding=1)
    for si, (nblocks, _mid, _cout, _stride) in enumerate(STAGES):
        for bi in range(nblocks):
            p = f"layer{si + 1}.{bi}"
            identity = x
            if bi == 0:
                identity = _ref_conv_bn(params, x, specs[p + ".down"], relu=False)
            y = _ref_conv_bn(params, x, specs[p + ".conv1"], relu=True)
            y = _ref_conv_bn(params, y, specs[p + ".conv2"], relu=True)
            x = _ref_conv_bn(params, y, specs[p + ".conv3"], relu=True, residual=identity)
    x = x.mean(dim=(2, 3))
    return F.linear(x, params["fc.w"], params["fc.b"])


class ResNet50Eager(torch.nn.Module):
    """Stock PyTorch-ROCm path (MIOpen convs), bf16 channels-last: comparison baseline (b).

    BN is kept as a separate op (as a user of stock PyTorch would run a torchvision model in
    eval mode); ``fold=True`` folds BN into the conv weights to give the eager path the same
    algorithmic advantage the fused path has.
    """

    def __init__(self, params: Dict[str, torch.Tensor], device, dtype=torch.bfloat16, fold: bool = True):
        super().__init__()
        self.specs = {s.name: s for s in conv_specs()}
        self.fold = fold
        self.dtype = dtype
        self.w: Dict[str, torch.Tensor] = {}
        self.sb: Dict[str, Tuple[torch.Tensor, torch.Tensor]] = {}
        for s in conv_specs():
            w = params[s.name + ".w"]
            scale, bias = fold_bn(params, s.name)
            if fold:
                w = w * scale.view(-1, 1, 1, 1)
            self.w[s.name] = w.to(device=device, dtype=dtype).contiguous(memory_format=torch.channels_last)
            self.sb[s.name] = (scale.to(device=device, dtype=dtype), bias.to(device=device, dtype=dtype))
        self.fc_w = params["fc.w"].to(device=device, dtype=dtype)
        self.fc_b = params["fc.b"].to(device=device, dtype=dtype)
        self.mean = torch.tensor(IMAGENET_MEAN, device=device, dtype=torch.float32)
        self.inv_std = 1.0 / torch.tensor(IMAGENET_STD, device=device, dtype=torch.float32)

    @torch.no_grad()
    def update_params(self, params: Dict[str, torch.Tensor]) -> None:
        """Hot weight reload, in place (see :meth:`ResNet50Fused.update_params`)."""
        for s in conv_specs():
            w = params[s.name + ".w"]
            scale, bias = fold_bn(params, s.name)
            if self.fold:
                w = w * scale.view(-1, 1, 1, 1)
            self.w[s.name].copy_(w)
            self.sb[s.name][0].copy_(scale)
            self.sb[s.name][1].copy_(bias)
        self.fc_w.copy_(params["fc.w"])
        self.fc_b.copy_(params["fc.b"])

    def _cbr(self, x, name, relu=True, residual=None):
        s = self.specs[name]
        y = F.conv2d(x, self.w[name], stride=s.stride, padding=s.pad)
        scale, bias = self.sb[name]
        if self.fold:
            y = y + bias.view(1, -1, 1, 1)
        else:
            y = y * scale.view(1, -1, 1, 1) + bias.view(1, -1, 1, 1)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y

    @torch.no_grad()
    def forward(self, images_u8_nhwc: torch.Tensor) -> torch.Tensor:
        x = ((images_u8_nhwc.float() - self.mean) * self.inv_std).to(self.dtype)
        x = x.permute(0, 3, 1, 2)  # NCHW view of NHWC memory == channels_last
        x = self._cbr(x, "stem")
        x = F.max_pool2d(x, 3, 2, 1)
        for si, (nblocks, _m, _c, _s) in enumerate(STAGES):
            for bi in range(nblocks):
                p = f"layer{si + 1}.{bi}"
                identity = self._cbr(x, p + ".down", relu=False) if bi == 0 else x
                y = self._cbr(x, p + ".conv1")
                y = self._cbr(y, p + ".conv2")
                x = self._cbr(y, p + ".conv3", residual=identity)
        x = x.mean(dim=(2, 3))
        return F.linear(x, self.fc_w, self.fc_b)


def conv_shapes(image_size: int = 224) -> List[Tuple[ConvSpec, int, int]]:
    """(spec, H_in, H_out) for every conv, in execution order (square images)."""
    out: List[Tuple[ConvSpec, int, int]] = []
    block_in = cur = image_size
    for s in conv_specs():
        if s.name.endswith(".conv1"):
            block_in = cur
        hin = block_in if s.name.endswith(".down") else cur
        ho = (hin + 2 * s.pad - s.k) // s.stride + 1
        out.append((s, hin, ho))
        if s.name == "stem":
            cur = (ho + 2 - 3) // 2 + 1  # maxpool 3x3/2 pad 1
        elif not s.name.endswith(".down"):
            cur = ho
    return out


def resnet50_flops_per_image(image_size: int = 224) -> float:
    """2*MACs of all convs + FC (BN folded away)."""
    total = 0.0
    for s, _hin, ho in conv_shapes(image_size):
        total += 2.0 * ho * ho * s.cout * s.cin * s.k * s.k
    return total + 2.0 * 2048 * NUM_CLASSES


class ResNet50Fused:
    """ResNet-50 on the hand-written CDNA4 kernels (``ops``), NHWC bf16, BN folded.

    Per conv: weights pre-multiplied by the BN scale (bf16, ``[Cout][KH][KW][Cin]``), the BN
    bias applied in fp32 in the GEMM epilogue together with the residual add and ReLU.  One
    split-K workspace per stream is shared by all layers (they run back-to-back on it), sized for
    ``max_batch`` and allocated at the first (eager) call on a stream, so nothing besides the
    activations is allocated inside a hipGraph capture (the capture's private pool owns those).

    ``tuning`` maps a layer name to an explicit ``(cfg, splitk)`` (see ``ops.autotune``);
    layers without an entry use the C++ heuristic.
    """

    def __init__(self, params: Dict[str, torch.Tensor], device, max_batch: int = 256,
                 tuning: Optional[Dict[str, Tuple[int, int]]] = None, image_size: int = 224):
        from .. import ops

        self.ops = ops
        self.device = torch.device(device)
        self.image_size = image_size
        self.tuning = dict(tuning or {})
        self.specs = {s.name: s for s in conv_specs()}
        self.w: Dict[str, torch.Tensor] = {}
        self.b: Dict[str, torch.Tensor] = {}
        for s in conv_specs():
            scale, bias = fold_bn(params, s.name)
            w = params[s.name + ".w"] * scale.view(-1, 1, 1, 1)
            self.w[s.name] = ops.pack_conv_weight(w).to(self.device)
            self.b[s.name] = bias.to(device=self.device, dtype=torch.float32).contiguous()
        # block 0 of each stage: conv3 + downsample projection as one GEMM over [y | x] (the identity
        # branch never goes to HBM): concatenated folded weights, summed biases
        self.dual_w: Dict[str, torch.Tensor] = {}
        self.dual_b: Dict[str, torch.Tensor] = {}
        for si, (_nb, _m, _c, _s) in enumerate(STAGES):
            p0 = f"layer{si + 1}.0"
            w3, wd = self.w[p0 + ".conv3"], self.w[p0 + ".down"]
            self.dual_w[p0] = torch.cat([w3.reshape(w3.shape[0], -1), wd.reshape(wd.shape[0], -1)], 1).contiguous()
            self.dual_b[p0] = (self.b[p0 + ".conv3"] + self.b[p0 + ".down"]).contiguous()
        self.fuse_down = True
        # conv3 -> next conv1 chaining at the layer1 / layer2 boundaries (csrc/conv_chain.hip);
        # MLS_CHAIN=0 runs the two convs as separate kernels
        self.chain = os.environ.get("MLS_CHAIN", "1") != "0"
        # block names whose conv3 is NOT chained (A/B: MLS_CHAIN_SKIP=layer1.2,layer2.1)
        self.chain_skip: set = {b for b in os.environ.get("MLS_CHAIN_SKIP", "").split(",") if b}
        # layer3 boundaries (K 256, N1 1024, N2 256): instantiated and tested, off by default --
        # interleaved A/B 51.3k vs 52.2k req/s with them (profiles/r2_chain_v2_ab.jsonl)
        self.chain_l3 = os.environ.get("MLS_CHAIN_L3", "0") == "1"
        if os.environ.get("MLS_CHAIN_L2_CW"):  # A/B: layer2 boundaries' chunk width (64 / 32)
            ops.set_chain_l2_cw(int(os.environ["MLS_CHAIN_L2_CW"]))
        if os.environ.get("MLS_CHAIN_L2_BM"):  # A/B: layer2 boundaries' row tile (128 / 64)
            ops.lib().mls_chain_set_l2_bm(int(os.environ["MLS_CHAIN_L2_BM"]))
        # normalise + stem + max pool as one kernel (csrc/stem_pool.hip); MLS_FUSED_STEM=0 -> 3 kernels
        self.fuse_stem = image_size == 224 and os.environ.get("MLS_FUSED_STEM", "1") != "0"
        # ... with layer1.0's 1x1 conv on the pooled tiles in the same kernel: tested, measured level
        # (51.3k vs 51.5k req/s, profiles/r2_stem_conv1_ab.jsonl), so opt-in (MLS_STEM_CONV1=1)
        self.fuse_stem_conv1 = os.environ.get("MLS_STEM_CONV1", "0") == "1"
        self.fc_w = params["fc.w"].to(device=self.device, dtype=torch.bfloat16).contiguous()
        self.fc_b = params["fc.b"].to(device=self.device, dtype=torch.float32).contiguous()
        self.num_classes = self.fc_w.shape[0]
        self.mean = IMAGENET_MEAN
        self.std = IMAGENET_STD
        self.max_batch = max_batch
        self._ws = ops.StreamWorkspace(self._workspace_bytes(max_batch) // 4 + 1, self.device)
        # fused head (MLS_FUSED_HEAD=0: avgpool + FC + softmax/top-k kernels): the last conv's
        # epilogue accumulates the global average pool into a per-stream fp32 buffer, one kernel
        # (csrc/head.hip) does FC + softmax + top-k and zeroes the buffer for the next forward
        self.fuse_head = os.environ.get("MLS_FUSED_HEAD", "1") != "0"
        self._pool = ops.StreamWorkspace(max_batch * self.fc_w.shape[1], self.device, zero=True)

    @property
    def workspace(self) -> torch.Tensor:
        return self._ws.get()

    @torch.no_grad()
    def update_params(self, params: Dict[str, torch.Tensor]) -> None:
        """Hot weight reload: fold / pack the new parameters and copy them INTO the existing device
        tensors, so every hipGraph already captured against them stays valid (no re-capture).
        The caller quiesces the engine first (no batch may read the weights mid-copy)."""
        from .. import ops

        for s in conv_specs():
            scale, bias = fold_bn(params, s.name)
            w = ops.pack_conv_weight(params[s.name + ".w"] * scale.view(-1, 1, 1, 1))
            self.w[s.name].copy_(w)
            self.b[s.name].copy_(bias)
        for si in range(len(STAGES)):
            p0 = f"layer{si + 1}.0"
            w3, wd = self.w[p0 + ".conv3"], self.w[p0 + ".down"]
            self.dual_w[p0].copy_(torch.cat([w3.reshape(w3.shape[0], -1), wd.reshape(wd.shape[0], -1)], 1))
            self.dual_b[p0].copy_(self.b[p0 + ".conv3"] + self.b[p0 + ".down"])
        self.fc_w.copy_(params["fc.w"])
        self.fc_b.copy_(params["fc.b"])

    # -- planning ---------------------------------------------------------------------------
    def layer_gemm_shapes(self, batch: int) -> List[Tuple[str, int, int, int]]:
        """(name, M, N, K) of every conv + the FC at ``batch``."""
        out = []
        for s, _hin, ho in conv_shapes(self.image_size):
            k = s.k * 32 if s.name == "stem" else s.k * s.k * s.cin
            out.append((s.name, batch * ho * ho, s.cout, k))
            if s.name.endswith(".0.down"):  # the fused conv3 + downsample GEMM of this block
                c3 = self.specs[s.name[: -len("down")] + "conv3"]
                out.append((s.name[: -len("down")] + "dual", batch * ho * ho, s.cout, c3.cin + s.cin))
        out.append(("fc", batch, self.num_classes, 2048))
        return out

    def _plan(self, name: str, M: int, N: int, K: int) -> Tuple[int, int]:
        if name in self.tuning:
            return self.tuning[name]
        return self.ops.gemm_heuristic(M, N, K)

    def _workspace_bytes(self, batch: int) -> int:
        need = 0
        for b in sorted({1, 2, 4, 8, 16, 32, 64, 128, 256, batch}):
            if b > batch:
                continue
            for name, M, N, K in self.layer_gemm_shapes(b):
                cfg, sk = self._plan(name, M, N, K)
                if cfg in self.ops.PIPE_CFGS:  # splitk = K split + 16 * (items per block - 1)
                    sk = sk % 16 or 1
                if sk > 1:
                    need = max(need, sk * M * N * 4)
        # the fused head's logits scratch
        return max(need, batch * NUM_CLASSES * 4, 1 << 20)

    # -- forward ----------------------------------------------------------------------------
    def _conv(self, x, name, act, residual=None, pad=None):
        s = self.specs[name]
        cfg, sk = self.tuning.get(name, (0, 0))
        return self.ops.conv2d_nhwc(x, self.w[name], self.b[name], kernel=s.k, stride=s.stride,
                                    pad=s.pad if pad is None else pad,
                                    residual=residual, act=act, workspace=self.workspace, cfg=cfg, splitk=sk)


    def _chained(self, p: str, nxt: str, dual: bool) -> bool:
        """Run block ``p``'s conv3 together with block ``nxt``'s conv1 (ops.conv1x1_chain)?"""
        if not self.chain or p in self.chain_skip:
            return False
        c3 = self.specs[p + ".conv3"]
        k = c3.cin + (self.specs[p + ".down"].cin if dual else 0)
        c1 = self.specs[nxt + ".conv1"]
        shape = (k, c3.cout, c1.cout)
        if shape == (256, 1024, 256) and not self.chain_l3:
            return False  # layer3: 49 tiles re-reading 1 MB of weights each -- measured slower (-3 %)
        return c1.k == 1 and c1.stride == 1 and shape in self.ops.CHAIN_SHAPES

    def forward(self, images_u8_nhwc: torch.Tensor) -> torch.Tensor:
        """uint8 ``[B,H,W,3]`` on device -> bf16 logits ``[B, num_classes]``."""
        ops = self.ops
        B = images_u8_nhwc.shape[0]
        if self.fuse_head:
            pooled = self._trunk(images_u8_nhwc, pool=True)
            _v, _i, logits = ops.fc_head(pooled, self.fc_w, self.fc_b, 0, logits=self._logits_buf(B))
            return logits.to(torch.bfloat16)
        x = self._trunk(images_u8_nhwc, pool=False)
        pooled = ops.avgpool_global_nhwc(x)
        cfg, sk = self.tuning.get("fc", (0, 0))
        return ops.gemm(pooled, self.fc_w, self.fc_b, workspace=self.workspace, cfg=cfg, splitk=sk)

    __call__ = forward

    def _logits_buf(self, B: int) -> torch.Tensor:
        return self.workspace[: B * self.num_classes].view(B, self.num_classes)

    def classify(self, images_u8_nhwc: torch.Tensor, k: int = 5, err: Optional[torch.Tensor] = None):
        """Head: logits -> softmax -> top-k.  Returns (probs fp32 [B,k], ids int32 [B,k]).  ``err``
        (int32 [B], ``ops.image_decode``'s per-image flags): flagged rows come back as ids -1 / NaN."""
        if self.fuse_head:
            pooled = self._trunk(images_u8_nhwc, pool=True)
            B = images_u8_nhwc.shape[0]
            vals, idx, _ = self.ops.fc_head(pooled, self.fc_w, self.fc_b, k, logits=self._logits_buf(B), err=err)
            return vals, idx
        vals, idx = self.ops.softmax_topk(self.forward(images_u8_nhwc), k)
        if err is not None:  # unfused A/B path: same contract, torch ops
            bad = (err[: idx.shape[0]] != 0).view(-1, 1)
            idx = torch.where(bad, torch.full_like(idx, -1), idx)
            vals = torch.where(bad, torch.full_like(vals, float("nan")), vals)
        return vals, idx

    def _trunk(self, images_u8_nhwc: torch.Tensor, pool: bool) -> torch.Tensor:
        """Stem .. layer4: the last block output ``[B,7,7,2048]`` bf16, or with ``pool`` its global
        average fp32 ``[B,2048]`` (fused into the last conv; the block output is never written)."""
        ops = self.ops
        B = images_u8_nhwc.shape[0]
        if B > self.max_batch:
            raise ValueError(f"batch {B} > max_batch {self.max_batch}")
        if self.fuse_stem and self.fuse_stem_conv1:  # + layer1.0.conv1 on each pooled tile
            x, t1 = ops.stem_pool_u8(images_u8_nhwc, self.w["stem"], self.b["stem"], self.mean, self.std,
                                     conv1_w=self.w["layer1.0.conv1"], conv1_b=self.b["layer1.0.conv1"])
        else:
            if self.fuse_stem:
                x = ops.stem_pool_u8(images_u8_nhwc, self.w["stem"], self.b["stem"], self.mean, self.std)
            else:
                x = ops.normalize_u8(images_u8_nhwc, self.mean, self.std, pad=3)  # zero border = stem padding
                x = self._conv(x, "stem", ops.ACT_RELU, pad=0)
                x = ops.maxpool2d_nhwc(x, 3, 2, 1)
            t1 = self._conv(x, "layer1.0.conv1", ops.ACT_RELU)
        blocks = [(si, bi) for si, (nblocks, _m, _c, _s) in enumerate(STAGES) for bi in range(nblocks)]
        for idx, (si, bi) in enumerate(blocks):
            p = f"layer{si + 1}.{bi}"
            nxt = f"layer{blocks[idx + 1][0] + 1}.{blocks[idx + 1][1]}" if idx + 1 < len(blocks) else None
            t2 = self._conv(t1, p + ".conv2", ops.ACT_RELU)
            dual = bi == 0 and self.fuse_down
            if nxt is not None and self._chained(p, nxt, dual):
                # this block's conv3 (+ residual / downsample) and the next block's conv1 in one
                # kernel: the block output goes to HBM once and is never read back
                w1n, b1n = self.w[nxt + ".conv1"], self.b[nxt + ".conv1"]
                w1n = w1n.reshape(w1n.shape[0], -1)
                if dual:
                    x, t1 = ops.conv1x1_chain(t2, self.dual_w[p], self.dual_b[p], w1n, b1n, a2=x,
                                              stride2=self.specs[p + ".down"].stride)
                else:
                    w3 = self.w[p + ".conv3"]
                    x, t1 = ops.conv1x1_chain(t2, w3.reshape(w3.shape[0], -1), self.b[p + ".conv3"], w1n, b1n,
                                              residual=x)
                continue
            if dual:
                cfg, sk = self.tuning.get(p + ".dual", (0, 0))
                x = ops.conv1x1_dual(t2, x, self.dual_w[p], self.dual_b[p], stride2=self.specs[p + ".down"].stride,
                                     act=ops.ACT_RELU, workspace=self.workspace, cfg=cfg, splitk=sk)
            else:
                identity = self._conv(x, p + ".down", ops.ACT_NONE) if bi == 0 else x
                if nxt is None and pool:  # the network's last conv: average pool in its epilogue
                    pooled = self._pool.get()[: B * self.fc_w.shape[1]].view(B, -1)
                    cfg, _sk = self.tuning.get(p + ".conv3", (0, 0))
                    s3 = self.specs[p + ".conv3"]
                    ops.conv2d_pool(t2, self.w[p + ".conv3"], self.b[p + ".conv3"], pooled, kernel=s3.k,
                                    stride=s3.stride, pad=s3.pad, residual=identity, act=ops.ACT_RELU, cfg=cfg)
                    return pooled
                x = self._conv(t2, p + ".conv3", ops.ACT_RELU, residual=identity)
            if nxt is not None:
                t1 = self._conv(x, nxt + ".conv1", ops.ACT_RELU)
        if pool:  # (the last block was a dual / chained one: not in ResNet-50, kept general)
            pooled = self._pool.get()[: B * self.fc_w.shape[1]].view(B, -1)
            pooled.copy_(ops.avgpool_global_nhwc(x).float())
            return pooled
        return x
