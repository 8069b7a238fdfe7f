"""Host timeline of the first submits after the bench's warm-up drain: where the ~0.5 ms before
the first batch's launch goes (bench.py's timed window starts with an idle pipeline)."""
import gc
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


def main():
    dev = torch.device("cuda:0")
    B = 32
    model = resnet.ResNet50Fused(resnet.init_resnet50(0), dev, max_batch=B, tuning=autotune.load_tuning("resnet50", B))
    ops.partition_masks(2, dev)
    eng = GpuEngine(lambda x: model.classify(x, 5), dev, (224, 224, 3), torch.uint8, buckets=[B], inflight=4,
                    concurrent=True, cu_partitions=2, name="probe")
    eng.warmup()
    rng = np.random.default_rng(0)
    pool = [[rng.integers(0, 256, (224, 224, 3), dtype=np.uint8) for _ in range(B)] for _ in range(4)]
    for rep in range(5):
        ts = [eng.submit(pool[i % 4]) for i in range(4)]
        [t.wait() for t in ts]
        torch.cuda.synchronize()
        gc.collect()
        gc.disable()
        time.sleep(0.001 * rep)
        marks = []
        t0 = time.perf_counter()
        tickets = []
        for i in range(4):
            a = time.perf_counter()
            slot = eng.acquire()
            b = time.perf_counter()
            eng._stager.gather(GpuEngine.host_buffer(slot), pool[i])
            c = time.perf_counter()
            tickets.append(eng.launch(slot, B))
            d = time.perf_counter()
            marks.append([round((x - t0) * 1e6, 1) for x in (a, b, c, d)])
        done = []
        for t in tickets:
            t.wait()
            done.append(round((time.perf_counter() - t0) * 1e6, 1))
        gc.enable()
        print(json.dumps({"rep": rep, "acquire_stage_launch_us": marks, "done_us": done}), flush=True)


if __name__ == "__main__":
    main()
