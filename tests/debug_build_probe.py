"""Run by test_debug_build_gpu.py in a child process with MLS_DEBUG=1 HIP_LAUNCH_BLOCKING=1:
legal calls pass the bounds checks, deliberate violations are reported (not faulted)."""
import sys

import torch

from mlmicroservicetemplate_amd import ops
from mlmicroservicetemplate_amd.ops import _lib
from mlmicroservicetemplate_amd.ops import reference as R

assert _lib.DEBUG and "debug" in ops.lib()._name, ops.lib()._name
dev = "cuda:0"
Hq, Hkv, D, B, ML = 8, 2, 128, 2, 256
kc = torch.randn(B, ML, Hkv, D, device=dev).to(torch.bfloat16)
vc = torch.randn_like(kc)
qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
cos, sin = R.rope_tables(ML, D, 500000.0, dev)
lens = torch.tensor([40, 200], device=dev, dtype=torch.int32)
pos = lens - 1
# legal
out = ops.decode_attention(qkv, kc, vc, lens, Hq, Hkv, D, positions=pos, cos=cos, sin=sin, max_len=256)
ref = R.decode_attention(qkv.clone(), kc, vc, lens, Hq, Hkv, D)  # (rope differs; only a smoke value check)
assert torch.isfinite(out.float()).all()
ops.rope_kv_(qkv.clone(), pos, cos, sin, Hq, Hkv, D, None, kc, vc, lens=lens, seq=1, max_seq=ML)
# violations
caught = []
try:
    ops.decode_attention(qkv, kc, vc, lens, Hq, Hkv, D, max_len=64)  # context bound below lens
except _lib.NativeError as e:
    caught.append(("201", str(e)))
try:
    bad = torch.tensor([0, 10 * ML], device=dev, dtype=torch.int32)
    ops.rope_kv_(qkv.clone(), torch.tensor([1, 2], device=dev, dtype=torch.int32), cos, sin, Hq, Hkv, D, bad, kc, vc)
except _lib.NativeError as e:
    caught.append(("101", str(e)))
try:
    ops.rope_kv_(qkv.clone(), torch.tensor([1, 5000], device=dev, dtype=torch.int32), cos, sin, Hq, Hkv, D, None,
                 kc, vc, lens=lens, seq=1, max_seq=ML)
except _lib.NativeError as e:
    caught.append(("102", str(e)))
codes = [c for c, _ in caught]
print(caught)
assert codes == ["201", "101", "102"], caught
# and the check state is clean afterwards
ops.decode_attention(qkv, kc, vc, lens, Hq, Hkv, D, max_len=256)
print("DEBUG-BUILD-OK")
sys.exit(0)
