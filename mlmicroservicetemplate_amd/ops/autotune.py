"""Per-shape tile/split-K autotuner for the implicit-GEMM conv / GEMM kernel (a "find" step).

For every ResNet-50 layer at a given batch, times each (tile cfg, split-K) candidate with
HIP events on random data and keeps the fastest; results are cached as JSON keyed by
(device arch, batch) so serving start-up does the search once per machine.  Also reports the
stock PyTorch-ROCm (MIOpen) time of the same conv for comparison.
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

CACHE_DIR = os.environ.get("MLS_TUNE_DIR", os.path.join(os.path.dirname(os.path.abspath(__file__)), "_native", "tune"))
GEMM_CFGS = list(range(1, 20)) + list(range(23, 32))  # conv_gemm.hip kCfgs (20..22: persistent kernel)
CANDIDATES: List[Tuple[int, int]] = [(c, s) for c in GEMM_CFGS for s in (1, 2, 4, 8)] + [(20, 1), (21, 1), (22, 1)]


def _flush_mb() -> int:
    """``MLS_TUNE_FLUSH_MB`` (default 0): after every timed call, a fill of that many MB (split over
    the co-running streams) evicts the L2s, so each call reads its operands from the MALL / HBM as a
    layer inside the forward does (its input was written by the previous kernel, often on other
    XCDs) instead of from an L2 warmed by the previous identical call; the fill's own time, measured
    alone, is subtracted."""
    return int(os.environ.get("MLS_TUNE_FLUSH_MB", "0"))


def _with_flush(fn, buf):
    def run():
        fn()
        buf.fill_(1)
    return run


def _time(fn, iters: int = 20, warmup: int = 3) -> float:
    """ms per call of ``fn`` measured on the GPU timeline: the ``iters`` calls are captured into
    one hipGraph and replayed, so host-side launch cost (Python + ctypes, ~10 us/call) cannot
    hide kernels shorter than it (timing eager launches would floor every kernel at that cost)."""
    mb = _flush_mb()
    if mb > 0:
        buf = torch.empty(mb << 20, dtype=torch.uint8, device=torch.cuda.current_device())
        t_fill = _time_plain(lambda: buf.fill_(1), iters, warmup)
        return max(_time_plain(_with_flush(fn, buf), iters, warmup) - t_fill, 0.0)
    return _time_plain(fn, iters, warmup)


def _time_plain(fn, iters: int = 20, warmup: int = 3) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warmup):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):  # the warm-up stream: its split-K counters exist
        for _ in range(iters):
            fn()
    g.replay()  # warm
    torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    start.record()
    g.replay()
    end.record()
    end.synchronize()
    del g
    return start.elapsed_time(end) / iters


_TUNE_STREAMS: list = []


def _time_multi(fns, iters: int = 20, warmup: int = 3) -> float:
    """ms per call when ``len(fns)`` independent copies of a layer co-run on their own streams
    (each captured in its own hipGraph): the per-call cost under the engine's concurrent slots,
    where a throughput-efficient tile beats a latency-optimal one."""
    if len(fns) == 1:
        return _time(fns[0], iters, warmup)
    mb = _flush_mb()
    if mb > 0:
        bufs = [torch.empty((mb << 20) // len(fns), dtype=torch.uint8, device=torch.cuda.current_device())
                for _ in fns]
        t_fill = _time_multi_plain([(lambda b=b: b.fill_(1)) for b in bufs], iters, warmup)
        return max(_time_multi_plain([_with_flush(f, b) for f, b in zip(fns, bufs)], iters, warmup) - t_fill, 0.0)
    return _time_multi_plain(fns, iters, warmup)


def _time_multi_plain(fns, iters: int = 20, warmup: int = 3) -> float:
    main = torch.cuda.current_stream()
    # MLS_TUNE_PARTITIONS=P: the copies run on CU-masked streams, copy i in partition i % P -- how a
    # partitioned serving engine (engine/worker.py, cu_partitions) co-runs its batches
    parts = int(os.environ.get("MLS_TUNE_PARTITIONS", "0"))
    masks = None
    if parts:
        from . import partition_masks

        masks = partition_masks(parts, main.device, mode=os.environ.get("MLS_CU_PARTITION_MODE", "intra"))
    if masks:
        from . import cu_masked_stream

        global _TUNE_STREAMS
        if len(_TUNE_STREAMS) < len(fns):  # masked streams are created once (each holds a hardware queue)
            _TUNE_STREAMS = [cu_masked_stream(masks[i % parts], main.device, key=i // parts) for i in range(len(fns))]
        streams = _TUNE_STREAMS[:len(fns)]
    else:
        streams = [torch.cuda.Stream() for _ in fns]
    graphs = []
    for fn, st in zip(fns, streams):
        st.wait_stream(main)
        with torch.cuda.stream(st):
            for _ in range(warmup):
                fn()
    torch.cuda.synchronize()
    for fn, st in zip(fns, streams):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(iters):
                fn()
        graphs.append(g)
    torch.cuda.synchronize()

    def replay_all():
        for g, st in zip(graphs, streams):
            st.wait_stream(main)
            with torch.cuda.stream(st):
                g.replay()
        for st in streams:
            main.wait_stream(st)

    replay_all()  # warm
    torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    start.record(main)
    replay_all()
    end.record(main)
    end.synchronize()
    del graphs
    return start.elapsed_time(end) / (iters * len(fns))


def tune_resnet50(batch: int, device="cuda:0", iters: int = 20, compare_torch: bool = True,
                  candidates: Optional[List[Tuple[int, int]]] = None, concurrency: int = 1,
                  layers: Optional[List[str]] = None) -> Dict[str, dict]:
    """Per-layer (cfg, splitk) search.  ``concurrency`` > 1 scores each candidate by its
    per-batch cost with that many batches co-running (the serving engine's concurrent slots).
    ``layers`` restricts the search to those layer names (probes); the FC is tuned only when
    ``layers`` is None or names it."""
    from . import CFG_HALO, CFG_HALO_N32, CFG_HALO_XL, CFG_PIPE, PIPE_VARIANTS, conv2d_nhwc, gemm, pack_conv_weight
    from ..models.resnet import conv_shapes

    dev = torch.device(device)
    ws = torch.empty(256 << 20, device=dev, dtype=torch.float32)
    results: Dict[str, dict] = {}
    cands = candidates or CANDIDATES
    for s, hin, ho in conv_shapes():
        if layers is not None and s.name not in layers:
            continue
        cin = 4 if s.name == "stem" else s.cin
        hp = hin + 2 * s.pad if s.name == "stem" else hin  # stem runs on the pre-padded image
        x = torch.randn(batch, hp, hp, cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(s.cout, s.cin, s.k, s.k, device=dev) * 0.05).to(torch.bfloat16)
        wp = pack_conv_weight(w)
        bias = torch.randn(s.cout, device=dev)
        res = torch.randn(batch, ho, ho, s.cout, device=dev).to(torch.bfloat16) if s.name.endswith("conv3") else None
        out = torch.empty(batch, ho, ho, s.cout, device=dev, dtype=torch.bfloat16)
        # per-stream copies for concurrent scoring (inputs shared read-only; outputs/scratch not)
        outs = [out] + [torch.empty_like(out) for _ in range(concurrency - 1)]
        wss = [ws] + [torch.empty_like(ws) for _ in range(concurrency - 1)]
        k = s.k * 32 if s.name == "stem" else s.k * s.k * s.cin
        flops = 2.0 * batch * ho * ho * s.cout * s.cin * s.k * s.k
        best = (1e9, 0, 0)
        tried = {}
        halo = s.k == 3 and s.stride == 1 and s.cin % 32 == 0 and s.cout % 64 == 0
        halo_cands = [(CFG_HALO, 1), (CFG_HALO, 2), (CFG_HALO, 4), (CFG_HALO_N32, 1), (CFG_HALO_XL, 1),
                      (CFG_HALO_XL, 2), (CFG_HALO_XL, 4)] if halo else []
        # the pipelined 3x3 kernel: variant x (K splits + 16 x (items per block - 1))
        pipe_cands = ([(CFG_PIPE + v, ks + 16 * (ipb - 1)) for v in range(PIPE_VARIANTS) for ks in (1, 2)
                       for ipb in (1, 2) if (s.cin // 32) % ks == 0] if halo and os.environ.get("MLS_TUNE_PIPE", "1") == "1"
                      else [])
        for cfg, sk in [(0, 0)] + cands + halo_cands + pipe_cands:
            if sk > 1 and cfg < CFG_PIPE and k // sk < 128:
                continue

            def mk(o, wsc, cfg=cfg, sk=sk):
                def run():
                    conv2d_nhwc(x, wp, bias, kernel=s.k, stride=s.stride, pad=0 if s.name == "stem" else s.pad,
                                residual=res, act=1, out=o, workspace=wsc, cfg=cfg, splitk=sk)
                return run

            try:
                t = _time_multi([mk(o, wsc) for o, wsc in zip(outs, wss)], iters)
            except Exception:  # e.g. split-K slabs beyond a per-stream scratch: not a candidate
                continue
            tried[f"{cfg},{sk}"] = round(t * 1e3, 2)
            if (cfg, sk) != (0, 0) and t < best[0]:
                best = (t, cfg, sk)
        print(f"autotune: {s.name} best cfg {best[1]} splitk {best[2]} {best[0] * 1e3:.2f} us "
              f"({len(tried)} tried)", file=sys.stderr, flush=True)  # progress (long GPU jobs)
        entry = {"M": batch * ho * ho, "N": s.cout, "K": k, "best_cfg": best[1], "best_splitk": best[2],
                 "best_us": round(best[0] * 1e3, 2), "heuristic_us": tried.get("0,0"),
                 "tflops": round(flops / (best[0] * 1e-3) / 1e12, 1)}
        if os.environ.get("MLS_TUNE_VERBOSE"):
            entry["tried_us"] = tried
        if compare_torch:
            xt = x[:, 3:-3, 3:-3, :3] if s.name == "stem" else x
            xt = xt.permute(0, 3, 1, 2)
            wt = w.contiguous(memory_format=torch.channels_last)
            bt = bias.to(torch.bfloat16).view(1, -1, 1, 1)

            def trun():
                y = F.conv2d(xt, wt, stride=s.stride, padding=s.pad) + bt
                return torch.relu(y)

            entry["torch_us"] = round(_time(trun, iters) * 1e3, 2)
        results[s.name] = entry
    # fused conv3 + downsample GEMMs (block 0 of each stage)
    from . import conv1x1_dual
    from ..models.resnet import STAGES

    shapes = {s.name: (s, hin, ho) for s, hin, ho in conv_shapes()}
    for si in range(len(STAGES)):
        p0 = f"layer{si + 1}.0"
        if layers is not None and p0 + ".dual" not in layers:
            continue
        sd, hin_d, ho = shapes[p0 + ".down"]
        s3 = shapes[p0 + ".conv3"][0]
        y = torch.randn(batch, ho, ho, s3.cin, device=dev).to(torch.bfloat16)
        xx = torch.randn(batch, hin_d, hin_d, sd.cin, device=dev).to(torch.bfloat16)
        wcat = (torch.randn(sd.cout, s3.cin + sd.cin, device=dev) * 0.05).to(torch.bfloat16)
        bias = torch.randn(sd.cout, device=dev)
        outs = [torch.empty(batch, ho, ho, sd.cout, device=dev, dtype=torch.bfloat16) for _ in range(concurrency)]
        wss = [ws] + [torch.empty_like(ws) for _ in range(concurrency - 1)]
        best = (1e9, 0, 0)
        tried = {}
        for cfg, sk in [(0, 0)] + cands:
            if 20 <= cfg <= 22:  # persistent kernel: no dual mode
                continue

            def mk(o, wsc, cfg=cfg, sk=sk):
                return lambda: conv1x1_dual(y, xx, wcat, bias, stride2=sd.stride, act=1, out=o, workspace=wsc,
                                            cfg=cfg, splitk=sk)

            try:
                t = _time_multi([mk(o, wsc) for o, wsc in zip(outs, wss)], iters)
            except Exception:
                continue
            tried[f"{cfg},{sk}"] = round(t * 1e3, 2)
            if (cfg, sk) != (0, 0) and t < best[0]:
                best = (t, cfg, sk)
        flops = 2.0 * batch * ho * ho * sd.cout * (s3.cin + sd.cin)
        results[p0 + ".dual"] = {"M": batch * ho * ho, "N": sd.cout, "K": s3.cin + sd.cin, "best_cfg": best[1],
                                 "best_splitk": best[2], "best_us": round(best[0] * 1e3, 2),
                                 "heuristic_us": tried.get("0,0"), "tflops": round(flops / (best[0] * 1e-3) / 1e12, 1)}
    if layers is not None and "fc" not in layers:
        return results
    # FC
    a = torch.randn(batch, 2048, device=dev).to(torch.bfloat16)
    w = torch.randn(1000, 2048, device=dev).to(torch.bfloat16)
    b = torch.randn(1000, device=dev)
    best = (1e9, 0, 0)
    for cfg, sk in cands:
        t = _time(lambda: gemm(a, w, b, workspace=ws, cfg=cfg, splitk=sk), iters)
        if t < best[0]:
            best = (t, cfg, sk)
    results["fc"] = {"M": batch, "N": 1000, "K": 2048, "best_cfg": best[1], "best_splitk": best[2],
                     "best_us": round(best[0] * 1e3, 2)}
    return results


def cache_path(batch: int) -> str:
    arch = "gfx950"
    try:
        arch = torch.cuda.get_device_properties(0).gcnArchName.split(":")[0]
    except Exception:
        pass
    return os.path.join(CACHE_DIR, f"resnet50_{arch}_b{batch}.json")


SHIPPED_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned")


def load_tuning(model: str, batch: int, arch: str = "gfx950", regime: str = "concurrent") -> Dict[str, Tuple[int, int]]:
    """Shipped (measured on MI355X, committed) or cached tuning table; {} -> C++ heuristic.
    ``regime``: "concurrent" -- the table measured under 4 co-running copies (the partitioned
    serving engine, the throughput bench); "serial" -- one batch alone on the chip (a one-slot engine,
    ``bench.py --serial``): ``<model>_<arch>_b<batch>_serial.json`` where shipped, where the
    pipelined 3x3 kernel wins every stride-1 3x3 (ResNet-50 serial forward 905-935 -> 815-820 us,
    ``profiles/r4_resnet50_serial_kernel_summary_*.txt``), else the concurrent table.
    ``MLS_TUNING_FILE`` overrides all (A/B runs of alternative tables)."""
    override = os.environ.get("MLS_TUNING_FILE")
    if override:
        with open(override) as f:
            data = json.load(f)
        return {k: (v["best_cfg"], v["best_splitk"]) for k, v in data.items()}
    names = [f"{model}_{arch}_b{batch}.json"]
    if regime == "serial":
        names.insert(0, f"{model}_{arch}_b{batch}_serial.json")
    for d, name in ((d, n) for n in names for d in (SHIPPED_DIR, CACHE_DIR)):
        path = os.path.join(d, name)
        if os.path.exists(path):
            with open(path) as f:
                data = json.load(f)
            return {k: (int(v["best_cfg"]), int(v["best_splitk"])) for k, v in data.items()}
    return {}


def load_or_tune(batch: int, device="cuda:0") -> Dict[str, Tuple[int, int]]:
    path = cache_path(batch)
    if os.path.exists(path):
        with open(path) as f:
            data = json.load(f)
    else:
        data = tune_resnet50(batch, device, compare_torch=False)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(data, f, indent=1)
    return {k: (v["best_cfg"], v["best_splitk"]) for k, v in data.items()}


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--out", default="")
    ap.add_argument("--concurrency", type=int, default=1)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--layers", nargs="*", default=None, help="only these layers (probe)")
    ap.add_argument("--cfgs", nargs="*", type=int, default=None, help="only these tile cfgs (with splitk 1/2/4/8)")
    ap.add_argument("--iters", type=int, default=20, help="graph-replayed calls per timing")
    args = ap.parse_args()
    t0 = time.time()
    cands = None
    if args.cfgs:
        cands = [(c, s) for c in args.cfgs for s in (1, 2, 4, 8)]
    res = tune_resnet50(args.batch, compare_torch=not args.no_torch, concurrency=args.concurrency,
                        candidates=cands, layers=args.layers, iters=args.iters)
    tot_best = sum(v["best_us"] for v in res.values())
    tot_heur = sum(v.get("heuristic_us") or v["best_us"] for v in res.values())
    tot_torch = sum(v.get("torch_us", 0) for v in res.values())
    for name, v in res.items():
        print(json.dumps({"layer": name, **v}))
    print(json.dumps({"sum_best_us": round(tot_best, 1), "sum_heuristic_us": round(tot_heur, 1),
                      "sum_torch_us": round(tot_torch, 1), "tune_s": round(time.time() - t0, 1)}))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
