"""Print the MAX_BATCH=0 capacity plan of the ResNet-50 plugin for a few latency SLOs."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mlmicroservicetemplate_amd.config import Settings  # noqa: E402
from mlmicroservicetemplate_amd.models import resnet  # noqa: E402
from mlmicroservicetemplate_amd.plugins.builtin import ResNet50Plugin  # noqa: E402

params = resnet.init_resnet50(0)
for slo in (2.0, 5.0, 20.0, 100.0):
    s = Settings.load(env_file=None, environ={}, overrides={"MAX_BATCH": 0, "LATENCY_SLO_MS": slo, "INFLIGHT": 5})
    p = ResNet50Plugin()
    p.plan_batch(s, "cuda:0", params)
    print(json.dumps({"slo_ms": slo, **p.capacity_plan.to_dict()}), flush=True)
