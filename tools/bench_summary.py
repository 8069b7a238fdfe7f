import sys, json
for l in open(sys.argv[1]):
    if '"metric"' not in l: continue
    r = json.loads(l)
    print(r["value"], r["p50_latency_ms"], r["p99_latency_ms"], r["steps"], r["config"]["inflight"])
