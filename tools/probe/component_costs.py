"""Per-component cost of the fused ResNet-50 forward (bs=32), graph-timed alone (c1) and with 4
copies co-running (c4, ~ the engine's steady state): stem, every conv / chain / dual call exactly as
ResNet50Fused.forward issues it (tuned cfgs), avgpool, FC, softmax-top-k.  Sum of c4 ~ ms per batch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mlmicroservicetemplate_amd import ops  # noqa: E402
from mlmicroservicetemplate_amd.models import resnet  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune  # noqa: E402


class Recorder:
    """Wraps the ops the forward calls; records (label, fn) closures with fresh outputs."""

    def __init__(self, model):
        self.model = model
        self.calls = []

    def run(self, imgs):
        real = {n: getattr(ops, n) for n in ("stem_pool_u8", "conv2d_nhwc", "conv1x1_chain", "conv1x1_dual",
                                              "avgpool_global_nhwc", "gemm", "softmax_topk")}
        rec = self

        def wrap(name):
            def f(*a, **k):
                out = real[name](*a, **k)
                rec.calls.append((name, a, k))
                return out
            return f

        for n in real:
            setattr(ops, n, wrap(n))
        try:
            with torch.no_grad():
                self.model.classify(imgs, 5)
        finally:
            for n, f in real.items():
                setattr(ops, n, f)
        return [(n, real[n], a, k) for n, a, k in self.calls]


def main():
    dev = torch.device("cuda:0")
    model = resnet.ResNet50Fused(resnet.init_resnet50(0), dev, max_batch=32,
                                 tuning=autotune.load_tuning("resnet50", 32))
    imgs = torch.randint(0, 256, (32, 224, 224, 3), dtype=torch.uint8, device=dev)
    calls = Recorder(model).run(imgs)
    tot = {1: 0.0, 4: 0.0}
    for i, (name, fn, a, k) in enumerate(calls):
        row = {"i": i, "op": name}
        for conc in (1, 4):
            wss = [torch.empty(64 << 20, device=dev, dtype=torch.float32) for _ in range(conc)]

            def mk(ws):
                kk = dict(k)
                if "workspace" in kk:
                    kk["workspace"] = ws
                for o in ("out", "y_out", "t1_out"):
                    kk.pop(o, None)
                return lambda: fn(*a, **kk)

            t = autotune._time_multi([mk(ws) for ws in wss], 20) * 1e3
            row[f"c{conc}_us"] = round(t, 2)
            tot[conc] += t
        print(json.dumps(row), flush=True)
    print(json.dumps({"sum_c1_us": round(tot[1], 1), "sum_c4_us": round(tot[4], 1), "calls": len(calls)}), flush=True)


if __name__ == "__main__":
    main()
