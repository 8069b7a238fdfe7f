"""In-forward tuner for the ResNet-50 per-layer conv tables: each candidate (cfg, splitk) of a layer
is scored by the time of the WHOLE captured forward with that layer switched, so a layer is judged
with its real inputs (written by the previous kernel, MALL-resident), its neighbours and -- in the
co-running regime -- the other batches it shares the CUs with.  ops.autotune times each layer alone
on an L2-hot input and misranks the latency-bound ones (docs/PERF_NOTES.md, round 5).

  REGIME=serial: one batch, back-to-back replays of its forward graph (per-forward time);
  REGIME=corun : 4 batches as the engine runs them, 2 per CU-masked half, replayed together
                 (time per round of 4 forwards).
Greedy in forward order; a switch is kept only if it beats the current pick by MIN_GAIN (0.4 %) in
an interleaved re-measurement.  Writes the updated table (shipped format) to --out."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models.resnet import ResNet50Fused, init_resnet50
    from mlmicroservicetemplate_amd.ops import autotune

    ap = argparse.ArgumentParser()
    ap.add_argument("--regime", default=os.environ.get("REGIME", "serial"), choices=["serial", "corun"])
    ap.add_argument("--layers", nargs="*", required=True)
    ap.add_argument("--splitk", type=int, nargs="*", default=[1, 2, 4])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--min-gain", type=float, default=0.004)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    regime = "serial" if a.regime == "serial" else "concurrent"
    table_path = os.path.join(autotune.SHIPPED_DIR, "resnet50_gfx950_b32" + ("_serial" if regime == "serial" else "") + ".json")
    table = json.load(open(table_path))
    model = ResNet50Fused(init_resnet50(0), dev, max_batch=32, tuning=autotune.load_tuning("resnet50", 32, regime=regime))
    if a.regime == "serial":
        streams = [torch.cuda.Stream(dev)]
    else:
        masks = ops.partition_masks(2, dev, mode="intra")
        assert masks, "CU masks not verified"
        streams = [ops.cu_masked_stream(masks[i % 2], dev, key=i // 2) for i in range(4)]
    xs = [torch.randint(0, 256, (32, 224, 224, 3), dtype=torch.uint8, device=dev) for _ in streams]

    def measure(reps=a.reps):
        """ms per round (one forward per stream) of freshly captured graphs."""
        with torch.no_grad():
            for x, s in zip(xs, streams):
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    model.classify(x, 5)
            torch.cuda.synchronize()
            gs = []
            for x, s in zip(xs, streams):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
                    model.classify(x, 5)
                gs.append(g)
            torch.cuda.synchronize()

            def rnd():
                for g, s in zip(gs, streams):
                    with torch.cuda.stream(s):
                        g.replay()

            for _ in range(3):
                rnd()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                rnd()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3 / reps
            del gs
        return dt

    cands_all = [(c, s) for c in autotune.GEMM_CFGS for s in a.splitk]
    base = measure()
    print(json.dumps({"regime": a.regime, "start_ms": round(base, 4)}), flush=True)
    for L in a.layers:
        cur = model.tuning.get(L, (0, 0))
        best, best_t = cur, base
        tried = 0
        for c in cands_all:
            if c == tuple(cur) or (L.endswith(".dual") and 20 <= c[0] <= 22):
                continue
            model.tuning[L] = c
            try:
                t = measure()
            except Exception:  # noqa: BLE001 -- unsupported combination
                continue
            tried += 1
            if t < best_t:
                best, best_t = c, t
        keep = cur
        if best != tuple(cur):  # confirm, interleaved
            tc, tb = [], []
            for _ in range(3):
                model.tuning[L] = cur
                tc.append(measure())
                model.tuning[L] = best
                tb.append(measure())
            if min(tb) < min(tc) * (1 - a.min_gain) and sorted(tb)[1] < sorted(tc)[1]:
                keep = best
                base = min(tb)
            else:
                base = min(tc)
        model.tuning[L] = keep
        print(json.dumps({"layer": L, "was": list(cur), "now": list(keep), "ms": round(base, 4), "tried": tried}),
              flush=True)
        if tuple(keep) != tuple(cur):
            e = dict(table.get(L, {}))
            e.update({"best_cfg": int(keep[0]), "best_splitk": int(keep[1]),
                      "note": f"in-forward tuned ({a.regime}: tools/inforward_tune.py)"})
            table[L] = e
    print(json.dumps({"regime": a.regime, "end_ms": round(base, 4)}), flush=True)
    with open(a.out, "w") as f:
        json.dump(table, f, indent=1)


if __name__ == "__main__":
    main()
