"""Child process for test_llama_tp_gpu.py: one TP rank of the fused (native-kernel) Llama; all
ranks share cuda:0 and talk over gloo (host-staged collectives)."""
import json
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mlmicroservicetemplate_amd.models.llama import GenParams, LlamaTP, TPComm, init_llama_shard, tiny_config

    cfg = tiny_config(**json.loads(os.environ["TP_CFG"]))
    p = init_llama_shard(cfg, world, rank, seed=3, device="cuda")
    m = LlamaTP(p, cfg, tp=world, rank=rank, comm=TPComm(None, world, device="cuda"), backend="fused",
                device="cuda", max_batch=4, max_seq=256)
    g = torch.Generator().manual_seed(7)
    ids = torch.randint(3, cfg.vocab - 1, (3, 24), generator=g)
    lens = torch.tensor([24, 11, 3])
    pos = torch.arange(24, dtype=torch.int32).unsqueeze(0).expand(3, 24).contiguous().cuda()
    vals, idx = m.step(ids.cuda(), pos, lens.cuda(), decode=False, k=8)
    allv = m.comm.all_gather(vals)
    alli = m.comm.all_gather(idx)
    # the overlapped TP prefill (two batch halves, all-reduces started early) vs the plain layer loop
    overlap_on = m.tp_overlap
    m.tp_overlap = False
    vals0, idx0 = m.step(ids.cuda(), pos, lens.cuda(), decode=False, k=8)
    m.tp_overlap = overlap_on
    overlap_diff = float((vals0.float() - vals.float()).abs().max())
    failed = ""
    stall_rank = int(os.environ.get("STALL_RANK", "-1"))
    if stall_rank >= 0:
        # fault injection: one rank's stream stalls past the peers' one-shot wait bound; every rank
        # must fail the request (TPCommError), not return tokens computed from partial sums
        from mlmicroservicetemplate_amd import ops
        from mlmicroservicetemplate_amd.models.llama import TPCommError

        # the prefill checks above ran with the default (~1 s) peer-wait bound: two ranks
        # time-sharing one GPU can miss a few-ms bound on any small all-reduce; only the stalled
        # request runs with the tight bound
        if m.comm.car is not None and os.environ.get("MLS_AR_TIMEOUT_ITERS_STALL"):
            m.comm.car.timeout = int(os.environ["MLS_AR_TIMEOUT_ITERS_STALL"])
        if rank == stall_rank:
            ops.gpu_sleep(int(os.environ.get("STALL_US", "300000")))
        try:
            m.generate(ids, lens, GenParams(max_new_tokens=8))
        except TPCommError as e:
            failed = type(e).__name__
    # count host round trips of the decode loop (.cpu() on device tensors)
    calls = []
    orig = torch.Tensor.cpu

    def counting_cpu(self, *a, **kw):
        if self.is_cuda:
            calls.append(tuple(self.shape))
        return orig(self, *a, **kw)

    torch.Tensor.cpu = counting_cpu
    try:
        out = m.generate(ids, lens, GenParams(max_new_tokens=8))
    finally:
        torch.Tensor.cpu = orig
    info = torch.tensor([int(m.use_graphs), int(m.comm.car is not None), len(m._graphs) + len(m._dev_graphs),
                         len(calls)])
    if m.comm.car is not None:
        info[1] += 10 * m.comm.car.errors()  # peer-wait timeouts would show here
    torch.save({"tokens": out.cpu(), "vals": allv.cpu(), "idx": alli.cpu(), "info": info, "failed": failed,
                "overlap_diff": overlap_diff},
               os.environ["OUT"] + f".{rank}.pt")
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
