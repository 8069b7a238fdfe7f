"""Per-launch boundary cost inside a captured hipGraph: a chain of N dependent tiny kernels replayed
(one-block and chip-wide grids), alone and with the ResNet forward's neighbours absent.  The cost per
launch here is the most that fusing launches can save per removed boundary (docs/PERF_NOTES.md,
round 6, "The persistent layer-3/4 bottleneck kernel")."""
import time

import torch


def chain_us(numel, n, reps=200):
    dev = torch.device("cuda:0")
    x = torch.zeros(numel, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        for _ in range(n):
            x.add_(1.0)
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6 / reps


def main():
    for numel, what in ((64, "1 block"), (256 * 1024, "~256 blocks"), (4 * 1024 * 1024, "~4k blocks (16 MB)")):
        t1, t45 = chain_us(numel, 1), chain_us(numel, 45)
        print(f"{what:22s} graph of 1 kernel {t1:7.2f} us, of 45 {t45:8.2f} us -> "
              f"{(t45 - t1) / 44:.2f} us per added dependent launch", flush=True)


if __name__ == "__main__":
    main()
