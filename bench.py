"""Flagship serving benchmark: ResNet-50 bs=32 requests/sec (whole node) + p50 latency.

BASELINE.json metric: "requests/sec (whole node) + p50 latency, ResNet-50 bs=32 at 1/2/4/8
MI355X".  One process per GPU; every rank is an independent
data-parallel serving replica (config 4 of BASELINE.json): rank 0 initialises the random
ResNet-50 weights and RCCL-broadcasts them over xGMI (X1), every rank builds its fused engine
and captures its hipGraph, then serves synthetic requests.

One timed *step* = one micro-batch of ``--batch`` requests through the full engine path:
per-request uint8 images (224x224x3) copied into a pinned staging slot -> H2D ->
hipGraph{normalise -> 53 fused MFMA convs -> pools -> FC -> softmax -> top-5} -> D2H of the
top-5 -> per-request numpy results.  ``--inflight`` batches are kept in flight per GPU, which
is how the server's batcher drives the engine.  Per-request latency = submit -> result.

Prints ONE JSON line on rank 0 (value = total requests/s over all ranks, computed from the
max elapsed time over ranks).  Weights are random-init and inputs synthetic (no network).

Launch modes:
  * ``python bench.py --gpus N`` with no ``WORLD_SIZE`` in the environment: this process is a
    pure launcher (it touches neither the GPU nor ``torch.cuda``) and starts N rank processes of
    itself (``parallel/launch.py``), relays rank 0's JSON line, and exits non-zero if any rank
    fails;
  * under ``torch.distributed.run`` (``WORLD_SIZE`` set): runs as that rank; ``--gpus`` must
    equal ``WORLD_SIZE`` or the bench refuses to run.
``MLS_DIST_BACKEND=gloo`` rehearses N ranks sharing fewer GPUs (RCCL refuses duplicate devices).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_model(backend: str, device, batch: int, params, serial: bool = False):
    import torch

    from mlmicroservicetemplate_amd.models import resnet

    if backend == "fused":
        from mlmicroservicetemplate_amd.ops import autotune

        # per-layer kernels measured for the regime the engine runs in: 4 co-running batches
        # (default) or one batch alone (--serial)
        tuning = autotune.load_tuning("resnet50", batch, regime="serial" if serial else "concurrent")
        model = resnet.ResNet50Fused(params, device, max_batch=batch, tuning=tuning)

        def fwd(x):
            return model.classify(x, 5)

    elif backend == "eager":
        model = resnet.ResNet50Eager(params, device, fold=True)

        def fwd(x):
            logits = model(x)
            v, i = torch.topk(torch.softmax(logits.float(), -1), 5, dim=-1)
            return v, i.to(torch.int32)

    else:
        raise ValueError(backend)
    return fwd


def agree_partitions(requested: int, local_ok: bool) -> int:
    """The CU-partition count every rank runs with: ``requested`` only if every rank's masks
    verified, else 0 on ALL ranks -- so one rank's fallback cannot leave the ranks running (and the
    JSON describing) different slot layouts."""
    from mlmicroservicetemplate_amd.parallel import dist as mdist

    return requested if mdist.all_ranks_true(bool(requested) and local_ok) else 0


def rank_config(local: dict) -> dict:
    """The per-rank engine settings (``local``) gathered over the process group and merged: agreed
    keys keep their value, disagreeing ones read ``"mixed"`` (``ranks_consistent`` false), plus the
    backend / world size the process group actually formed."""
    from mlmicroservicetemplate_amd.parallel import dist as mdist

    merged = mdist.merge_rank_configs(mdist.gather_objects(dict(local)))
    merged.update(mdist.group_description())
    return merged


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--inflight", type=int, default=int(os.environ.get("INFLIGHT", 0)),
                    help="batches in flight per GPU (0 = 4 with CU partitions, else 5)")
    ap.add_argument("--cu-partition", type=int, default=int(os.environ.get("MLS_CU_PARTITION", 2)),
                    help="spatial partitions of the CUs for the in-flight batches (engine/worker.py; 0 = off)")
    ap.add_argument("--backend", default="fused", choices=["fused", "eager"])
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--serial", action="store_true", help="one compute stream (no concurrent in-flight batches)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--measure-eager", type=int, default=int(os.environ.get("MLS_MEASURE_EAGER", 20)),
                    metavar="STEPS",
                    help="after the timed run (which it does not touch), time STEPS batches of the "
                         "stock-PyTorch (MIOpen/hipBLASLt) engine in the same process and report "
                         "vs_pytorch_eager_per_gpu -- BASELINE.md's config-2 bar; 0 = skip")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="launcher mode: bound on the whole N-rank job (s)")
    return ap.parse_args(argv)


def launch_ranks(args, argv) -> int:
    """Launcher mode: N rank processes of this script, rank 0's JSON relayed (no GPU touched here)."""
    from mlmicroservicetemplate_amd.parallel.launch import spawn_ranks

    cmd = [sys.executable, "-u", os.path.abspath(__file__), *argv]
    log(f"bench: launching {args.gpus} ranks")
    return spawn_ranks(cmd, args.gpus, timeout_s=args.launch_timeout)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus < 1:
        log("--gpus must be >= 1")
        return 2
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args, argv)
    if env_world is not None and int(env_world) != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={env_world}; refusing to report a mislabelled run")
        return 2
    return run_rank(args)


def run_rank(args) -> int:
    import numpy as np
    import torch

    from mlmicroservicetemplate_amd.parallel import dist as mdist

    info = mdist.init_distributed()
    world = info.world_size
    # one GPU per rank; with fewer visible GPUs than ranks (a gloo rehearsal on a 1-GPU box,
    # MLS_DIST_BACKEND=gloo) ranks share them round-robin
    ndev = max(1, torch.cuda.device_count())
    device = torch.device("cuda", info.local_rank % ndev)
    torch.cuda.set_device(device)
    from mlmicroservicetemplate_amd.parallel.affinity import bind_to_gpu

    numa_cpus = bind_to_gpu(device.index, world)  # host staging on the GPU's NUMA node

    from mlmicroservicetemplate_amd.engine.worker import GpuEngine
    from mlmicroservicetemplate_amd.models import resnet

    # ---- X1: rank 0 initialises, everyone receives over RCCL (not timed) ----
    t0 = time.perf_counter()
    params = resnet.init_resnet50(args.seed) if info.rank == 0 else None
    if world > 1:
        spec = {k: (tuple(v.shape), v.dtype) for k, v in resnet.init_resnet50_spec().items()}
        params = mdist.broadcast_state(params, src=0, device=device, spec=spec)
        torch.cuda.synchronize(device)  # X1 done before any graph capture starts
    t_bcast = time.perf_counter() - t0

    fwd = build_model(args.backend, device, args.batch, params, serial=args.serial)
    if args.serial:
        args.cu_partition = 0
    if args.cu_partition:
        from mlmicroservicetemplate_amd import ops

        # the census-verified masks (cached for the engine); a device whose mask layout does not
        # verify runs unpartitioned -- and then with the 5 slots of that mode
        local_ok = ops.partition_masks(args.cu_partition, device,
                                       mode=os.environ.get("MLS_CU_PARTITION_MODE", "intra")) is not None
        if not local_ok:
            print(f"bench: CU partitions unavailable on {device}; unpartitioned", file=sys.stderr)
    else:
        local_ok = False
    # every rank runs the same layout: one rank without verified masks takes all ranks unpartitioned
    agreed = agree_partitions(args.cu_partition, local_ok) if world > 1 else (args.cu_partition if local_ok else 0)
    if agreed != args.cu_partition and local_ok:
        print(f"bench: rank {info.rank}: another rank cannot partition its CUs; all ranks unpartitioned",
              file=sys.stderr)
    args.cu_partition = agreed
    if args.inflight <= 0:
        args.inflight = 4 if args.cu_partition and not args.serial else 5
    # MLS_BENCH_PRESTAGE=1: the next batch is staged into a spare pinned buffer (GpuEngine.prepare)
    # while every slot is busy, so a freed slot only waits for the enqueue -- how a server stages
    # requests as they arrive; the slot's graph pulls it straight from that buffer
    # (ops.h2d_pull_cell).  Request latency then runs from the start of its staging
    # (Ticket.t_arrive), not from the launch.  Level at 20 steps, -1 % at 200, p50 +0.27 ms
    # (profiles/r6_bench_prestage_prepull_ab.jsonl): off by default
    prestage = os.environ.get("MLS_BENCH_PRESTAGE", "0") == "1"
    # the closed-loop client polls its oldest batch's done event (20 ms bound) instead of sleeping
    # in a blocking sync: s200 56.0k vs 55.2k req/s (profiles/r5_stall_ab_sdma_vs_pull.jsonl)
    engine = GpuEngine(fwd, device, (224, 224, 3), torch.uint8, buckets=[args.batch], inflight=args.inflight,
                       use_graphs=not args.no_graphs, name=f"resnet50.r{info.rank}", concurrent=not args.serial,
                       cu_partitions=0 if args.serial else args.cu_partition, spin_wait_us=20000.0)
    cu_parts = engine.cu_partitions
    engine.warmup(capture=not args.no_graphs)
    # what every rank actually runs (the engine itself can still fall back, e.g. no hardware queue
    # left for a masked stream): merged over the ranks, "mixed" where they disagree
    ranks_cfg = rank_config({
        "backend": args.backend, "hipgraph": not args.no_graphs, "inflight": args.inflight,
        "concurrent_slots": not args.serial, "cu_partitions": cu_parts,
        "partition_mode": (os.environ.get("MLS_CU_PARTITION_MODE", "intra") if cu_parts else "unpartitioned"),
        "prestage": prestage, "batch": args.batch, "numa_bound": bool(numa_cpus)})
    if not ranks_cfg["ranks_consistent"]:
        print(f"bench: ranks disagree on the engine layout: {ranks_cfg}", file=sys.stderr)

    rng = np.random.default_rng(1234 + info.rank)
    pool = [[rng.integers(0, 256, (224, 224, 3), dtype=np.uint8) for _ in range(args.batch)] for _ in range(4)]

    host_s = [0.0]  # host time spent inside submit() (staging copy + enqueue): diagnostics

    tickets_log = os.environ.get("MLS_BENCH_TICKETS")  # diagnostics: per-batch submit / done times
    events: list = []


    # MLS_BENCH_WAIT_ANY=1: refill from whichever in-flight batch completes first (polling their
    # done events) instead of the oldest -- how a server's batcher refills a freed slot
    wait_any = os.environ.get("MLS_BENCH_WAIT_ANY", "0") == "1"

    def oldest_or_first_done(pending):
        if not wait_any:
            return 0
        while True:
            for k, t in enumerate(pending):
                if t.slot.ev_done.query():
                    return k

    def run_steps(n, lat):
        pending = []
        nxt = engine.prepare(pool[0]) if prestage and n else None
        for i in range(n):
            t0 = time.perf_counter()
            if prestage:
                pending.append(engine.launch_prepared(nxt))
                if i + 1 < n:
                    nxt = engine.prepare(pool[(i + 1) % len(pool)])
            else:
                pending.append(engine.submit(pool[i % len(pool)]))
            host_s[0] += time.perf_counter() - t0
            if len(pending) >= args.inflight:
                t = pending.pop(oldest_or_first_done(pending))
                t.wait()
                lat.append(time.perf_counter() - t.t_arrive)
                events.append((t.t_arrive, time.perf_counter(), getattr(t, "stamps", None),
                               getattr(t, "launch_ns", None)))
        for t in pending:
            t.wait()
            lat.append(time.perf_counter() - t.t_arrive)
            events.append((t.t_arrive, time.perf_counter(), getattr(t, "stamps", None),
                           getattr(t, "launch_ns", None)))

    phases = os.environ.get("MLS_BENCH_PHASES")  # diagnostics: wall-clock stamps of the phases

    def stamp(what):
        if phases and info.rank == 0:
            with open(phases, "a") as f:
                f.write(f"{what} {time.time():.3f}\n")

    # no cyclic-GC pass inside the ~13 ms window (a full collection over torch's object graph is
    # milliseconds of host time the submit loop would stall for; the servers gc.freeze() their
    # start-up objects once the model is ready: api/app.py, frontend/native.py).  The collection
    # runs BEFORE the warmup steps: collected between them and the window, its idle gap left the
    # window's first submit cold (staging 0.16 vs 0.09 ms, graph launch 67-94 vs 28-53 us) and the
    # 20-step value 2.6 % lower (5 of 5 interleaved pairs, profiles/r5_s20_gc_before_warmup_ab.jsonl)
    gc.collect()
    gc.disable()
    # The warmup is the W requested steps AND at least MLS_BENCH_WARM_MS (default 200) of
    # continuous serving: from idle (graph capture, the collection above) the GPU needs tens of ms
    # of load to reach its serving clocks, and W = 5 steps are ~3 ms -- the 20-step window then ran
    # ~5 % below the same tree's steady state (52.2-52.7k vs 54.8-55.6k with a 50-200 ms floor, 3 of 3
    # interleaved pairs each; a floor placed before the collection did not help: the idle gap
    # loses it; profiles/r6_bench_warmup_floor_ab.jsonl).  Untimed like the W steps; the timed K
    # steps are unchanged, and the warmed 20-step value stays below the 200-step one.
    warm_floor_ms = float(os.environ.get("MLS_BENCH_WARM_MS", "200"))
    warm_steps = [0]

    def warm_up(n):
        tw = time.perf_counter()
        run_steps(n, [])
        warm_steps[0] += n
        while (time.perf_counter() - tw) * 1e3 < warm_floor_ms:
            run_steps(2 * args.inflight, [])
            warm_steps[0] += 2 * args.inflight
        return (time.perf_counter() - tw) * 1e3

    stamp("warmup")
    warm_ms = warm_up(args.warmup)
    warm_n = warm_steps[0]
    host_s[0] = 0.0
    events.clear()
    lat: list = []
    mdist.barrier()
    torch.cuda.synchronize(device)
    stamp("timed")
    t_start = time.perf_counter()
    run_steps(args.steps, lat)
    torch.cuda.synchronize(device)
    mdist.barrier()
    elapsed = time.perf_counter() - t_start
    gc.enable()
    stamp("done")
    if tickets_log and info.rank == 0:
        with open(tickets_log, "a") as f:
            f.write(json.dumps({"steps": args.steps, "elapsed_ms": elapsed * 1e3,
                                "tickets_ms": [[round((a - t_start) * 1e3, 3), round((b - t_start) * 1e3, 3)]
                                               for a, b, _, _ in events],
                                # per submit: slot wait, staging, enqueue (ms)
                                "submit_phases_ms": [None if st is None else
                                                     [round((st[i + 1] - st[i]) * 1e3, 3) for i in range(3)]
                                                     for _, _, st, _ in events],
                                # per native enqueue: H2D copy, graph launch, D2H copies, event (us)
                                "launch_us": [None if ln is None else [round(x / 1e3, 1) for x in ln]
                                              for _, _, _, ln in events]}) + "\n")
    elapsed_max = mdist.max_over_ranks(elapsed)
    p50 = float(np.percentile(lat, 50)) * 1e3
    p99 = float(np.percentile(lat, 99)) * 1e3
    p50_max = mdist.max_over_ranks(p50)
    p99_max = mdist.max_over_ranks(p99)
    # per-rank req/s and p50 (each rank's own clock), in rank order
    per_rank = mdist.gather_objects((round(args.batch * args.steps / elapsed, 1), round(p50, 3)))
    host_ms = host_s[0] * 1e3 / args.steps
    host_ms_max = mdist.max_over_ranks(host_ms)  # the slowest rank's host side
    from mlmicroservicetemplate_amd.parallel.affinity import host_plan_hint

    plan = host_plan_hint()

    total_req = world * args.batch * args.steps
    value = total_req / elapsed_max
    eager = None
    if args.measure_eager > 0:  # stock-PyTorch engine, same process / box / protocol (not the flagship)
        efwd = build_model("eager", device, args.batch, params)
        eeng = GpuEngine(efwd, device, (224, 224, 3), torch.uint8, buckets=[args.batch], inflight=args.inflight,
                         use_graphs=not args.no_graphs, name=f"eager.r{info.rank}", concurrent=not args.serial,
                         cu_partitions=0 if args.serial else args.cu_partition, spin_wait_us=20000.0)
        eeng.warmup(capture=not args.no_graphs)
        engine = eeng
        warm_up(min(args.warmup, 5))  # the same warmup floor as the flagship's
        mdist.barrier()
        torch.cuda.synchronize(device)
        te = time.perf_counter()
        run_steps(args.measure_eager, [])
        torch.cuda.synchronize(device)
        mdist.barrier()
        eager = mdist.max_over_ranks(time.perf_counter() - te)
        eager = args.batch * args.measure_eager / eager
    if info.rank == 0:
        out = {
            "metric": "requests/sec (whole node) + p50 latency, ResNet-50 bs=32",
            "value": round(value, 1),
            "unit": "requests/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_ms": round(warm_ms, 1),  # W steps, then more untimed steps up to MLS_BENCH_WARM_MS
            "warmup_steps_run": warm_n,
            "ms_per_step": round(elapsed_max * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic uint8 224x224x3 images, random-init weights",
            # the slot layout every rank ran (CU-masked partitions with 4 slots, or the unpartitioned
            # 5-slot fallback), merged over the ranks: "mixed" + ranks_consistent false if they differ
            "config": {"model": "resnet50-v1.5", "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "seq_len": None, "image_size": 224, "parallelism": f"dp{world}",
                       **{k: v for k, v in ranks_cfg.items() if k != "batch"}},
            "p50_latency_ms": round(p50_max, 3),
            "p99_latency_ms": round(p99_max, 3),
            "per_gpu_requests_per_s": round(value / world, 1),
            "per_rank_requests_per_s": [v for v, _ in per_rank],
            "per_rank_p50_latency_ms": [p for _, p in per_rank],
            **({"pytorch_eager_per_gpu_requests_per_s": round(eager, 1),
                "vs_pytorch_eager_per_gpu": round(value / world / eager, 3)} if eager else {}),
            "weight_broadcast_s": round(t_bcast, 3),
            "host_submit_ms_per_step": round(host_ms, 4),
            **({"host_submit_ms_per_step_max_rank": round(host_ms_max, 4),
                "host_plan_rank0": plan} if world > 1 else {}),
        }
        print(json.dumps(out), flush=True)
    mdist.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
