"""Re-score every 3x3 / stride-1 layer of the shipped ResNet-50 bs=32 tuning table with the halo
kernel as an extra candidate (ops.CFG_HALO), under the same 4-way co-running timing the table was
tuned with; writes the updated table + a per-layer comparison (JSONL) to gpurun_out/."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mlmicroservicetemplate_amd import ops  # noqa: E402
from mlmicroservicetemplate_amd.models.resnet import conv_shapes  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune  # noqa: E402

CONC = int(os.environ.get("CONC", "4"))
dev = torch.device("cuda:0")
path = os.path.join(autotune.SHIPPED_DIR, "resnet50_gfx950_b32.json")
with open(path) as f:
    table = json.load(f)
B = 32
for s, hin, ho in conv_shapes():
    if not (s.k == 3 and s.stride == 1 and s.name in table):
        continue
    x = torch.randn(B, hin, hin, s.cin, device=dev).to(torch.bfloat16)
    wp = ops.pack_conv_weight((torch.randn(s.cout, s.cin, 3, 3, device=dev) * 0.05).to(torch.bfloat16))
    bias = torch.randn(s.cout, device=dev)
    outs = [torch.empty(B, ho, ho, s.cout, device=dev, dtype=torch.bfloat16) for _ in range(CONC)]
    wss = [torch.empty(64 << 20, device=dev, dtype=torch.float32) for _ in range(CONC)]
    ent = table[s.name]
    res = {}
    cur = (ent["best_cfg"], ent["best_splitk"])
    cands = [cur, (ops.CFG_HALO, 1), (ops.CFG_HALO_N32, 1)]
    for cfg, sk in dict.fromkeys(cands):
        fns = [lambda o=o, w_=w_, cfg=cfg, sk=sk: ops.conv2d_nhwc(x, wp, bias, kernel=3, stride=1, pad=1, act=1, out=o,
                                                                  workspace=w_, cfg=cfg, splitk=sk)
               for o, w_ in zip(outs, wss)]
        res[(cfg, sk)] = autotune._time_multi(fns, 20) * 1e3
    (cfg, sk), us = min(res.items(), key=lambda kv: kv[1])
    print(json.dumps({"layer": s.name, "concurrency": CONC, "table_cfg": list(cur), "table_us": round(res[cur], 2),
                      "halo64_us": round(res[(ops.CFG_HALO, 1)], 2), "halo32_us": round(res[(ops.CFG_HALO_N32, 1)], 2),
                      "chosen": [cfg, sk]}), flush=True)
    if (cfg, sk) != cur:
        ent.update(best_cfg=cfg, best_splitk=sk, best_us=round(us, 2),
                   tflops=round(2.0 * B * ho * ho * s.cout * s.cin * 9 / (us * 1e-3) / 1e12, 1))
os.makedirs("gpurun_out", exist_ok=True)
with open("gpurun_out/resnet50_gfx950_b32_halo.json", "w") as f:
    json.dump(table, f, indent=1)
