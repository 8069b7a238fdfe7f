"""Phase stamps of the v2 stem kernel (csrc/stem_pool.hip, mls_stem_set_stamps): per wave, s_memtime at
the start, after the first loads, and around each tile's patch write / MFMAs / epilogue / pool.
Prints the median cycles of each phase over all waves, and the block start / end spread."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlmicroservicetemplate_amd import ops  # noqa: E402
from mlmicroservicetemplate_amd.models.resnet import IMAGENET_MEAN, IMAGENET_STD  # noqa: E402

dev = torch.device("cuda:0")
B = 32
imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
wp = ops.pack_conv_weight((torch.randn(64, 3, 7, 7, device=dev) * 0.05).to(torch.bfloat16))
bias = torch.randn(64, device=dev)
out = torch.empty(B, 56, 56, 64, device=dev, dtype=torch.bfloat16)
for _ in range(5):
    ops.stem_pool_u8(imgs, wp, bias, IMAGENET_MEAN, IMAGENET_STD, out=out)
torch.cuda.synchronize()
st = torch.zeros(B * 16 * 4 * 64, dtype=torch.int64, device=dev)
ops.lib().mls_stem_set_stamps(st.data_ptr())
for _ in range(3):
    ops.stem_pool_u8(imgs, wp, bias, IMAGENET_MEAN, IMAGENET_STD, out=out)
torch.cuda.synchronize()
ops.lib().mls_stem_set_stamps(None)
s = st.view(B * 16 * 4, 64).cpu().double()
T = 7
med = lambda x: float(x.median())  # noqa: E731
res = {"waves": s.shape[0], "kernel_span": float(s[:, 2 + 6 * T].max() - s[:, 0].min()),
       "start_spread": float(s[:, 0].max() - s[:, 0].min()), "first_loads": med(s[:, 1] - s[:, 0]),
       "wave_total": med(s[:, 2 + 6 * T] - s[:, 0])}
names = ["barrier1", "patch", "barrier2", "mfma", "epi+barrier3", "pool"]
for t in range(T):
    b0 = 1 if t == 0 else 7 + 6 * (t - 1)
    cols = [b0, 2 + 6 * t, 3 + 6 * t, 4 + 6 * t, 5 + 6 * t, 6 + 6 * t, 7 + 6 * t]
    res[f"t{t}"] = {n: med(s[:, cols[i + 1]] - s[:, cols[i]]) for i, n in enumerate(names)}
print(json.dumps(res), flush=True)
