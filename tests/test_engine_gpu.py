"""GpuEngine on MI355X: concurrent in-flight slots (per-slot streams + graph pools, per-stream
split-K workspace) must give exactly the results of one-at-a-time execution."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_concurrent_slots_match_serial():
    from mlmicroservicetemplate_amd.engine.worker import GpuEngine
    from mlmicroservicetemplate_amd.models import resnet
    from mlmicroservicetemplate_amd.ops.autotune import load_tuning

    p = resnet.init_resnet50(0)
    model = resnet.ResNet50Fused(p, DEV, max_batch=8, tuning=load_tuning("resnet50", 8))

    def fwd(x):
        v, i = model.classify(x, 5)
        return v, i

    rng = np.random.default_rng(0)
    batches = [rng.integers(0, 256, (8, 224, 224, 3), dtype=np.uint8) for _ in range(6)]
    serial = GpuEngine(fwd, DEV, (224, 224, 3), torch.uint8, buckets=[8], inflight=1, name="serial")
    serial.warmup()
    ref = [serial.run(b) for b in batches]
    conc = GpuEngine(fwd, DEV, (224, 224, 3), torch.uint8, buckets=[8], inflight=3, concurrent=True, name="conc")
    conc.warmup()
    assert conc.stats()["concurrent"]
    for _ in range(3):
        # keep three batches in flight: each submit beyond the third waits for a free slot, so
        # the oldest ticket is collected first
        pending, outs = [], []
        for b in batches:
            if len(pending) == 3:
                outs.append(pending.pop(0).wait())
            pending.append(conc.submit(b))
        outs += [t.wait() for t in pending]
        for (rv, ri), (ov, oi) in zip(ref, outs):
            np.testing.assert_array_equal(ri, oi)
            np.testing.assert_array_equal(rv, ov)
