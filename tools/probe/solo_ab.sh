# Solo launches (a lone batch on the whole GPU) in the partitioned engine: tests, one-at-a-time
# latency, bench A/B.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/solo
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 - > $OUT/latency.jsonl 2> $OUT/lat.err <<'PY' || { tail -20 $OUT/lat.err; exit 1; }
import json, os, time, numpy as np, torch
from mlmicroservicetemplate_amd.engine.worker import GpuEngine
from mlmicroservicetemplate_amd.models import resnet
from mlmicroservicetemplate_amd.ops.autotune import load_tuning
model = resnet.ResNet50Fused(resnet.init_resnet50(0), "cuda:0", max_batch=32, tuning=load_tuning("resnet50", 32))
b = np.random.default_rng(0).integers(0, 256, (32, 224, 224, 3), dtype=np.uint8)
for name, parts, solo in (("unpartitioned", 0, "1"), ("partitioned_solo", 2, "1"), ("partitioned_masked", 2, "0")):
    os.environ["MLS_SOLO_FULL"] = solo
    eng = GpuEngine(lambda x: model.classify(x, 5), "cuda:0", (224, 224, 3), torch.uint8, buckets=[32], inflight=4,
                    concurrent=True, name=name, cu_partitions=parts)
    eng.warmup()
    for _ in range(5): eng.run(b)
    lat = []
    for _ in range(50):
        t = time.perf_counter(); eng.run(b); lat.append(time.perf_counter() - t)
    lat.sort()
    print(json.dumps({"engine": name, "one_batch_at_a_time_p50_ms": round(lat[25] * 1e3, 3),
                      "p90_ms": round(lat[45] * 1e3, 3), "solo_launches": eng.solo_launches}), flush=True)
PY
cat $OUT/latency.jsonl
for r in 1 2; do for solo in 1 0; do
  MLS_SOLO_FULL=$solo timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/b20_${solo}_$r.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  MLS_SOLO_FULL=$solo timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 > $OUT/b200_${solo}_$r.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "solo=$solo r=$r s20 $(python3 -c "import json; d=json.load(open('$OUT/b20_${solo}_$r.json')); print(d['value'], d['p50_latency_ms'])") s200 $(python3 -c "import json; d=json.load(open('$OUT/b200_${solo}_$r.json')); print(d['value'], d['p50_latency_ms'])")"
done; done
