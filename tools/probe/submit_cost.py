"""Host cost of one engine submit on the flagship config (ResNet-50 bs=32, partitioned engine):
staging copy vs the enqueue (H2D + graph replay + D2H + events), and the bare hipGraph replay call.
One JSON line per phase (median / p90 over the calls, microseconds of host time)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mlmicroservicetemplate_amd import ops  # noqa: E402
from mlmicroservicetemplate_amd.engine.worker import GpuEngine  # noqa: E402
from mlmicroservicetemplate_amd.models import resnet  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune  # noqa: E402


def stats(name, xs):
    xs = np.array(xs) * 1e6
    print(json.dumps({"phase": name, "n": len(xs), "median_us": round(float(np.median(xs)), 1),
                      "p90_us": round(float(np.percentile(xs, 90)), 1)}), flush=True)


def main():
    dev = torch.device("cuda:0")
    B = 32
    model = resnet.ResNet50Fused(resnet.init_resnet50(0), dev, max_batch=B, tuning=autotune.load_tuning("resnet50", B))
    ops.partition_masks(2, dev)
    eng = GpuEngine(lambda x: model.classify(x, 5), dev, (224, 224, 3), torch.uint8, buckets=[B], inflight=4,
                    concurrent=True, cu_partitions=2, name="probe")
    eng.warmup()
    rng = np.random.default_rng(0)
    imgs = [rng.integers(0, 256, (224, 224, 3), dtype=np.uint8) for _ in range(B)]
    stage, launch, wait = [], [], []
    for it in range(60):
        t0 = time.perf_counter()
        slot = eng.acquire()
        eng._stager.gather(GpuEngine.host_buffer(slot), imgs)
        t1 = time.perf_counter()
        tk = eng.launch(slot, B)
        t2 = time.perf_counter()
        tk.wait()
        t3 = time.perf_counter()
        if it >= 10:
            stage.append(t1 - t0)
            launch.append(t2 - t1)
            wait.append(t3 - t2)
    stats("stage_gather", stage)
    stats("launch_enqueue", launch)
    stats("wait_one_batch_alone", wait)
    slot = eng.slots[0]
    g = slot.graphs[B]
    torch.cuda.synchronize()
    rep = []
    for it in range(40):
        with torch.cuda.stream(slot.s_comp):
            t0 = time.perf_counter()
            g.replay()
            rep.append(time.perf_counter() - t0)
        slot.s_comp.synchronize()
    stats("graph_replay_call", rep[5:])
    print(json.dumps({"graph_nodes": None}), flush=True)


if __name__ == "__main__":
    main()
