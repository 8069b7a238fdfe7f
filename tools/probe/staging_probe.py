"""Host staging copy rate into a pinned slot: native pool vs Python threads, 1-8 threads.
One ResNet-50 batch (32 x 224x224x3 uint8 = 4.8 MB) per call; prints one JSON line per config."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlmicroservicetemplate_amd.engine.staging import HostStager  # noqa: E402

rng = np.random.default_rng(0)
pool = [[rng.integers(0, 256, (224, 224, 3), dtype=np.uint8) for _ in range(32)] for _ in range(4)]
dst = torch.zeros((32, 224, 224, 3), dtype=torch.uint8, pin_memory=True).numpy()
for native in (True, False):
    for th in (1, 2, 4, 6, 8):
        st = HostStager(th, native=native)
        for i in range(10):
            st.gather(dst, pool[i % 4])
        t = time.perf_counter()
        for i in range(300):
            st.gather(dst, pool[i % 4])
        dt = (time.perf_counter() - t) / 300
        print(json.dumps({"native": native, "threads": th, "ms_per_batch": round(dt * 1e3, 4),
                          "GBps": round(32 * 150528 / dt / 1e9, 2)}), flush=True)
