"""Where the engine's ~11 % over a bare replay loop goes (docs/PERF_NOTES.md, round 5): 4 forwards
co-running on the 2 CU-masked halves, replayed in rounds, with and without the engine's graph-resident
I/O kernels (ops.h2d_pull of the pinned uint8 batch before the forward, ops.d2h_push of the top-5
after it), interleaved in one process.  What is left between this and the bench is host-side (the
closed loop's refill of a slot after its batch completes)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models.resnet import ResNet50Fused, init_resnet50
    from mlmicroservicetemplate_amd.ops import autotune

    dev = torch.device("cuda:0")
    model = ResNet50Fused(init_resnet50(0), dev, max_batch=32, tuning=autotune.load_tuning("resnet50", 32))
    masks = ops.partition_masks(2, dev, mode="intra")
    assert masks
    ss = [ops.cu_masked_stream(masks[i % 2], dev, key=i // 2) for i in range(4)]
    xs = [torch.randint(0, 256, (32, 224, 224, 3), dtype=torch.uint8, device=dev) for _ in ss]
    hs = [x.cpu().pin_memory() for x in xs]
    outs = [torch.empty(32, 5, dtype=torch.float32).pin_memory() for _ in ss]

    def build(io):
        gs = []
        with torch.no_grad():
            for i, s in enumerate(ss):
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    model.classify(xs[i], 5)
            torch.cuda.synchronize()
            for i, s in enumerate(ss):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
                    if io:
                        ops.h2d_pull(hs[i], xs[i], blocks=8)
                    v = model.classify(xs[i], 5)
                    if io:
                        vals = v[0] if isinstance(v, (tuple, list)) else v
                        ops.d2h_push(vals.float().contiguous(), outs[i])
                gs.append(g)
            torch.cuda.synchronize()
        return gs

    def run(gs, reps=60):
        def rnd():
            for g, s in zip(gs, ss):
                with torch.cuda.stream(s):
                    g.replay()
        for _ in range(5):
            rnd()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            rnd()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / reps / len(gs)

    # hidden pull: per stream two input buffers; graph k (forward of buffer k + push) is replayed while
    # a masked side stream of the same half pulls the next batch into the other buffer (what an engine
    # fed by more batches than slots could do); the compute stream waits on the pull's event
    xs2 = [torch.empty_like(x) for x in xs]
    # SIDE=masked: the side streams on the same half's mask; SIDE=plain: ordinary (unmasked) streams
    if os.environ.get("SIDE", "masked") == "plain":
        sides = [torch.cuda.Stream(dev) for _ in range(4)]
    else:
        sides = [ops.cu_masked_stream(masks[i % 2], dev, key=2 + i // 2) for i in range(4)]

    def build_fwd(bufs):
        gs = []
        with torch.no_grad():
            for i, s in enumerate(ss):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
                    v = model.classify(bufs[i], 5)
                    vals = v[0] if isinstance(v, (tuple, list)) else v
                    ops.d2h_push(vals.float().contiguous(), outs[i])
                gs.append(g)
            torch.cuda.synchronize()
        return gs

    g0, g1 = build(False), build(True)  # (their eager warm-up allocates the per-stream head scratch)
    ga, gb = build_fwd(xs), build_fwd(xs2)

    # SYNC=event (default): side stream + event waits; none: no waits (timing only); same: the pull
    # on the slot's own stream after its graph (in-order, no cross-stream dependency)
    SYNC = os.environ.get("SYNC", "event")

    def run_hidden(reps=60):
        def rnd(k):
            gs, nxt = (ga, xs2) if k % 2 == 0 else (gb, xs)
            for i, (g, s, sd) in enumerate(zip(gs, ss, sides)):
                if SYNC == "none":  # timing only (races the buffers): no cross-stream wait at all
                    with torch.cuda.stream(sd):
                        ops.h2d_pull(hs[i], nxt[i], blocks=8)
                    with torch.cuda.stream(s):
                        g.replay()
                    continue
                if SYNC == "same":  # the pull as a separate launch on the slot's own stream (no cross-stream)
                    with torch.cuda.stream(s):
                        g.replay()
                        ops.h2d_pull(hs[i], nxt[i], blocks=8)
                    continue
                ev = torch.cuda.Event()
                with torch.cuda.stream(sd):
                    sd.wait_stream(s)  # the buffer it overwrites was read by the graph before last
                    ops.h2d_pull(hs[i], nxt[i], blocks=8)
                    ev.record(sd)
                with torch.cuda.stream(s):
                    g.replay()
                    s.wait_event(ev)  # the next round's graph reads the pulled buffer
        for k in range(6):
            rnd(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(reps):
            rnd(k)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / reps / len(ss)

    for r in range(3):
        a, b, c = run(g0), run(g1), run_hidden()
        print(f"round {r}: ms per batch  no-IO {a:.4f}  with pull+push {b:.4f}  (+{100 * (b / a - 1):.1f} %)  "
              f"pull on a side stream, next batch {c:.4f}  (+{100 * (c / a - 1):.1f} %)", flush=True)


if __name__ == "__main__":
    main()
