"""Child process for test_custom_ar_gpu.py: rank r of a gloo group whose ranks all drive cuda:0
(one GPU box); exercises the IPC one-shot all-reduce eagerly and inside a captured hipGraph."""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mlmicroservicetemplate_amd.parallel.custom_ar import CustomAllReduce

    dev = torch.device("cuda:0")
    car = CustomAllReduce(None, dev, cap_bytes=1 << 20, cap2_bytes=4 << 20, two_shot_min=128 << 10)
    assert car.enabled, car.reason
    g = torch.Generator().manual_seed(rank)
    fails = 0
    paths = set()
    # one-shot sizes, then two-shot ones (>= 128 KiB, multiples of 8 x world)
    for n in (8, 4096, 4104, 65536, 300000, 8 * world * 8192, 256 * 4096, 8 * world * 25003):
        x = torch.randn(n, generator=g).to(torch.bfloat16)
        ref = x.float().clone()
        dist.all_reduce(ref)
        paths.add(car.path(x.to(dev)))
        y = car.all_reduce_(x.to(dev))
        torch.cuda.synchronize()
        err = (y.float().cpu() - ref).abs().max().item() / ref.abs().max().item()
        fails += err > 2e-2
        # every rank holds the same bytes (one reducer per element)
        yy = y.float().cpu()
        first = yy.clone()
        dist.broadcast(first, 0)
        fails += int(not torch.equal(first, yy))
    fails += int(paths != {"one_shot", "two_shot"})
    # two-shot inside a captured graph as well (256 decode rows x 4096 hidden = 2 MiB)
    big = torch.zeros(256 * 4096, device=dev, dtype=torch.bfloat16)
    s2 = torch.cuda.Stream(dev)
    with torch.cuda.stream(s2):
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=s2):
            car.all_reduce_(big)
    for it in range(3):
        big.copy_(torch.full((256 * 4096,), float(rank + it), dtype=torch.bfloat16).to(dev))
        torch.cuda.synchronize()
        dist.barrier()
        g2.replay()
        torch.cuda.synchronize()
        fails += int(not torch.all(big.float() == sum(r + it for r in range(world))).item())
    # captured in a graph: three all-reduces per replay, replayed twice (device-side epochs)
    bufs = [torch.zeros(4096, device=dev, dtype=torch.bfloat16) for _ in range(3)]
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for b in bufs:
                car.all_reduce_(b)
    for it in range(2):
        vals = [torch.full((4096,), float(rank + 1 + i + it), dtype=torch.bfloat16) for i in range(3)]
        for b, v in zip(bufs, vals):
            b.copy_(v.to(dev))
        torch.cuda.synchronize()
        dist.barrier()
        graph.replay()
        torch.cuda.synchronize()
        for i, b in enumerate(bufs):
            want = sum(r + 1 + i + it for r in range(world))
            fails += int(not torch.all(b.float() == want).item())
    # GEMM-fused all-reduce (ops.skinny_packed_ar): each rank's x_r @ W_r^T summed over the ranks in
    # the GEMM's own epilogue; interleaved with standalone one-shot calls (shared per-chunk epochs),
    # eagerly and inside a captured graph
    from mlmicroservicetemplate_amd import ops

    gw = torch.Generator().manual_seed(100 + rank)
    for M, N, K in ((1, 4096, 512), (3, 768, 256), (8, 4096, 1792), (4, 2048, 512)):
        x = (torch.randn(M, K, generator=gw) * 0.5).to(torch.bfloat16)
        w = (torch.randn(N, K, generator=gw) / K ** 0.5).to(torch.bfloat16)
        ref = x.float() @ w.float().T
        dist.all_reduce(ref)
        wp = ops.pack_skinny(w.to(dev))
        xd = x.to(dev)
        for rep in range(2):
            y = ops.skinny_packed_ar(xd, wp, N, car)
            torch.cuda.synchronize()
            err = (y.float().cpu() - ref).abs().max().item() / ref.abs().max().item()
            fails += err > 2e-2
            if err > 2e-2:
                print(f"rank {rank} fused M={M} N={N} K={K} rep={rep} err={err}", flush=True)
            z = car.all_reduce_(torch.ones(4096, device=dev, dtype=torch.bfloat16))  # standalone in between
            torch.cuda.synchronize()
            fails += int(not torch.all(z.float() == world).item())
    # captured: fused GEMM + standalone one-shot in one graph, replayed
    x = (torch.randn(2, 512, generator=gw) * 0.5).to(torch.bfloat16)
    w = (torch.randn(4096, 512, generator=gw) / 512 ** 0.5).to(torch.bfloat16)
    ref = x.float() @ w.float().T
    dist.all_reduce(ref)
    wp, xd = ops.pack_skinny(w.to(dev)), x.to(dev)
    yo = torch.empty(2, 4096, device=dev, dtype=torch.bfloat16)
    z = torch.empty(4096, device=dev, dtype=torch.bfloat16)
    s3 = torch.cuda.Stream(dev)
    with torch.cuda.stream(s3):
        g3 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g3, stream=s3):
            ops.skinny_packed_ar(xd, wp, 4096, car, out=yo)
            car.all_reduce_(z)
    for it in range(3):
        z.fill_(float(rank + it))
        torch.cuda.synchronize()
        dist.barrier()
        g3.replay()
        torch.cuda.synchronize()
        err = (yo.float().cpu() - ref).abs().max().item() / ref.abs().max().item()
        fails += err > 2e-2
        fails += int(not torch.all(z.float() == sum(r + it for r in range(world))).item())
    fails += car._errors()
    # a peer lost before a GEMM-fused all-reduce: the fused kernel's peer waits honour
    # CustomAllReduce.timeout (not a built-in ~1 s per chunk), a block that timed out on one chunk
    # does not spin the full bound again on its next ones, and the error word reports it
    import time

    x = (torch.randn(8, 1792, generator=gw) * 0.5).to(torch.bfloat16).to(dev)
    wp = ops.pack_skinny((torch.randn(4096, 1792, generator=gw) / 1792 ** 0.5).to(torch.bfloat16).to(dev))
    torch.cuda.synchronize()
    dist.barrier()
    car.timeout = 20000
    t0 = time.perf_counter()
    if rank == world - 1:
        ops.gpu_sleep(1500000)  # the "lost" peer arrives 1.5 s late
    ops.skinny_packed_ar(x, wp, 4096, car)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if rank != world - 1:
        err = car._errors()
        print(f"rank {rank} fused stall: {dt * 1e3:.1f} ms, error word {err}", flush=True)
        fails += int(err == 0) + int(dt > 1.0)
    dist.barrier()
    car._errors()
    car.reset()
    car.timeout = 1 << 24
    y = ops.skinny_packed_ar(xd, ops.pack_skinny(w.to(dev)), 4096, car)  # the protocol works again
    torch.cuda.synchronize()
    fails += int((y.float().cpu() - ref).abs().max().item() / ref.abs().max().item() > 2e-2)
    fails += car._errors()
    car.close()
    dist.destroy_process_group()
    print(f"rank {rank} fails {fails}")
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
