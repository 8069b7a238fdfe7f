"""Per-layer kernel times of the fused ResNet-50 forward as the engine runs it: 4 batches co-running,
2 on each CU-masked half (``ops.partition_masks(2, mode="intra")``), each replaying its captured
forward graph back to back.  Run under ``rocprofv3 --kernel-trace``; ``--report <db>`` then prints the
mean duration of the i-th kernel of a forward over every stream and replay (queue_id tells the
streams apart).  MLS_TUNING_FILE selects the table under test."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run():
    import torch

    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models.resnet import ResNet50Fused, init_resnet50
    from mlmicroservicetemplate_amd.ops import autotune

    dev = torch.device("cuda:0")
    iters = int(os.environ.get("ITERS", "20"))
    model = ResNet50Fused(init_resnet50(0), dev, max_batch=32,
                          tuning=autotune.load_tuning("resnet50", 32, regime="concurrent"))
    masks = ops.partition_masks(2, dev, mode="intra")
    assert masks, "CU masks not verified on this box"
    ss = [ops.cu_masked_stream(masks[i % 2], dev, key=i // 2) for i in range(4)]
    xs = [torch.randint(0, 256, (32, 224, 224, 3), dtype=torch.uint8, device=dev) for _ in ss]
    gs = []
    with torch.no_grad():
        for x, s in zip(xs, ss):
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                model.classify(x, 5)
        torch.cuda.synchronize()
        for x, s in zip(xs, ss):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
                model.classify(x, 5)
            gs.append(g)
        torch.cuda.synchronize()
        for _ in range(iters):
            for g, s in zip(gs, ss):
                with torch.cuda.stream(s):
                    g.replay()
        torch.cuda.synchronize()
    print("corun forwards", iters, "x", len(ss), flush=True)


def report(db):
    import collections
    import sqlite3

    rows = sorted(sqlite3.connect(db).execute("select queue_id, start, end, name from kernels").fetchall(),
                  key=lambda r: r[1])
    per_q = collections.defaultdict(list)
    for q, s, e, n in rows:
        per_q[q].append((s, e, n))
    seqs = []
    for q, ks in per_q.items():  # split each queue's kernels into forwards at the stem kernel
        cur = None
        for s, e, n in ks:
            if "stem" in n:
                if cur:
                    seqs.append(cur)
                cur = []
            if cur is not None:
                cur.append((e - s, n))
    lens = collections.Counter(len(q) for q in seqs)
    L = lens.most_common(1)[0][0]  # the captured forward's kernel count (warm-up forwards differ)
    seqs = [q for q in seqs if len(q) == L]
    tot = 0.0
    for i in range(L):
        d = sum(q[i][0] for q in seqs) / len(seqs) / 1e3
        tot += d
        n = seqs[0][i][1].replace("void ", "").replace("(anonymous namespace)::", "")
        print(f"{i:3d} {d:8.2f}  {n[:n.find('(')] if '(' in n else n}"[:100])
    print(f"sum of kernel means {tot:.1f} us over {len(seqs)} forwards")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run()
