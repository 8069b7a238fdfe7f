# NUMA binding check on the box: bench with binding forced vs off, and the 2-rank gloo rehearsal
set -o pipefail
mkdir -p gpurun_out
python -c "import torch;from mlmicroservicetemplate_amd.parallel.affinity import pci_address,gpu_local_cpus;a=pci_address(0);print(a, len(gpu_local_cpus(a) or []))" > gpurun_out/numa_probe.log 2>&1 && \
MLS_NUMA_BIND=1 timeout -k 10 200 python bench.py > gpurun_out/bench_numa1.log 2>&1 && \
MLS_NUMA_BIND=0 timeout -k 10 200 python bench.py > gpurun_out/bench_numa0.log 2>&1 && \
MLS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 100 --warmup 10 > gpurun_out/bench_2rank_gloo.log 2>&1
