"""Run one GEMM shape through a few impls (for rocprofv3 --pmc passes): IMPLS env = comma list of
blas / tile<cfg>; each impl runs ITERS times after a warm-up."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlmicroservicetemplate_amd import ops  # noqa: E402

M, N, K = (int(x) for x in os.environ.get("SHAPE", "8192,8192,8192").split(","))
iters = int(os.environ.get("ITERS", "5"))
dev = torch.device("cuda")
x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
for impl in os.environ.get("IMPLS", "blas,tile1").split(","):
    if impl == "blas":
        fn = lambda: torch.mm(x, w.t())  # noqa: E731
    else:
        cfg = int(impl[4:])
        fn = lambda c=cfg: ops.gemm_tile(x, w, cfg=c)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
print("ok")
