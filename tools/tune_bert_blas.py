"""Offline PyTorch TunableOp search for the BERT-base projection GEMMs at larger batch buckets
(B x S rows = 8192 / 16384: the dynamic batcher's 64 / 128 buckets at S = 128).  Runs the fused
BERT forward eagerly with tuning on, so exactly the GEMM calls the engine makes (bias, GELU
epilogue, layouts) are tuned, then writes the new solutions to --out (append them to
ops/tuned/tunableop_gfx950.csv; tuning stays off at run time -- lookup only).

    python tools/tune_bert_blas.py --batches 64 128 --out gpurun_out/bert_tuned.csv
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[64, 128])
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    from torch.cuda import tunable

    from mlmicroservicetemplate_amd.models import bert

    dev = torch.device("cuda:0")
    cfg = bert.BertConfig()
    model = bert.BertFused(bert.init_bert(cfg, 0), dev, cfg)
    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_filename(args.out)
    tunable.set_max_tuning_duration(60)  # ms of timing per solution candidate set
    for B in args.batches:
        g = torch.Generator().manual_seed(B)
        ids = torch.randint(1000, 30000, (B, args.seq), generator=g, dtype=torch.int32).to(dev)
        tt = torch.zeros_like(ids)
        lens = torch.full((B,), args.seq, dtype=torch.int32, device=dev)
        t0 = time.time()
        with torch.no_grad():
            model.classify(ids, tt, lens, 2)
        torch.cuda.synchronize()
        print(f"tuned B={B} S={args.seq} in {time.time() - t0:.1f}s", flush=True)
    # the results file is written when the process exits (TunableOp's own flush)
    for r in tunable.get_results():
        print(r, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
