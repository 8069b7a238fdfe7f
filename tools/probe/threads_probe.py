import threading, sys, os
sys.path.insert(0, os.getcwd())
import bench
args = bench.parse_args(["--steps", "1", "--warmup", "1", "--measure-eager", "0"])
import torch
from mlmicroservicetemplate_amd.parallel import dist as mdist
info = mdist.init_distributed()
print("after init_distributed", [(t.name, t.daemon) for t in threading.enumerate()], flush=True)
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
from mlmicroservicetemplate_amd.parallel.affinity import bind_to_gpu
bind_to_gpu(0, 1)
from mlmicroservicetemplate_amd.engine.worker import GpuEngine
from mlmicroservicetemplate_amd.models import resnet
params = resnet.init_resnet50(0)
fwd = bench.build_model("fused", dev, 32, params)
from mlmicroservicetemplate_amd import ops
ops.partition_masks(2, dev)
eng = GpuEngine(fwd, dev, (224, 224, 3), torch.uint8, buckets=[32], inflight=4, concurrent=True, cu_partitions=2)
eng.warmup()
print("after engine", [(t.name, t.daemon) for t in threading.enumerate()], flush=True)
print("switchinterval", sys.getswitchinterval())
