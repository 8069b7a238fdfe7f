"""HTTP load generator for ``POST /predict`` (T11 of SURVEY.md §1.2).

Closed loop (``--concurrency C`` clients, each sends its next request when the previous one
returns) or open loop (``--rate R`` requests/s, Poisson arrivals).  Payload: raw RGB8
224x224x3 (``application/octet-stream``, skips JPEG decode on the server) or a synthetic JPEG
(``--jpeg``).  ``--spawn MODEL`` starts the service itself (e.g. ``identity`` on CPU for
config 1) and stops it afterwards.  Prints one JSON line: req/s, p50/p90/p99 latency, errors.
"""
from __future__ import annotations

import argparse
import asyncio
import io
import json
import os
import random
import signal
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mlmicroservicetemplate_amd.api.multipart import encode_multipart  # noqa: E402


def make_payload(jpeg: bool, seed: int = 0):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (224, 224, 3), dtype=np.uint8)
    if jpeg:
        from PIL import Image

        buf = io.BytesIO()
        Image.fromarray(img).resize((320, 240)).save(buf, format="JPEG", quality=90)
        return encode_multipart({"image_file": ("img.jpg", buf.getvalue(), "image/jpeg")})
    return encode_multipart({"image_file": ("img.rgb", img.tobytes(), "application/octet-stream")})


async def run(url: str, duration: float, concurrency: int, rate: float, payloads, warmup: float):
    import aiohttp

    lat = []
    errors = 0
    codes = {}
    t_end = time.perf_counter() + warmup + duration
    t_measure = time.perf_counter() + warmup
    conn = aiohttp.TCPConnector(limit=0, force_close=False)
    async with aiohttp.ClientSession(connector=conn) as sess:

        async def one(i):
            nonlocal errors
            body, ct = payloads[i % len(payloads)]
            t0 = time.perf_counter()
            try:
                async with sess.post(url, data=body, headers={"content-type": ct}) as r:
                    await r.read()
                    codes[r.status] = codes.get(r.status, 0) + 1
                    ok = r.status == 200
            except Exception:
                ok = False
            t1 = time.perf_counter()
            if t0 >= t_measure:
                if ok:
                    lat.append(t1 - t0)
                else:
                    errors += 1

        if rate > 0:
            tasks = set()
            i = 0
            nxt = time.perf_counter()
            while time.perf_counter() < t_end:
                now = time.perf_counter()
                if now < nxt:
                    await asyncio.sleep(nxt - now)
                t = asyncio.create_task(one(i))
                tasks.add(t)
                t.add_done_callback(tasks.discard)
                i += 1
                nxt += random.expovariate(rate)
            if tasks:
                await asyncio.gather(*tasks)
        else:
            async def client(cid):
                i = cid
                while time.perf_counter() < t_end:
                    await one(i)
                    i += concurrency

            await asyncio.gather(*[client(c) for c in range(concurrency)])
    return lat, errors, codes


def _client_proc(url, duration, concurrency, rate, jpeg, warmup, seed):
    payloads = [make_payload(jpeg, 8 * seed + s) for s in range(8)]
    return asyncio.run(run(url, duration, concurrency, rate, payloads, warmup))


def wait_ready(base: str, timeout: float = 600) -> bool:
    import requests

    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            if requests.get(base + "/status", timeout=2).status_code == 200:
                return True
        except Exception:
            pass
        time.sleep(0.5)
    return False


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--url", default="http://127.0.0.1:5005")
    ap.add_argument("--duration", type=float, default=10.0)
    ap.add_argument("--warmup", type=float, default=2.0)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--rate", type=float, default=0.0, help="open-loop req/s (0 = closed loop)")
    ap.add_argument("--jpeg", action="store_true")
    ap.add_argument("--spawn", default="", help="start the service with this MODEL first")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--max-batch", type=int, default=32)
    ap.add_argument("--extra", default="", help="extra args for the spawned server")
    ap.add_argument("--procs", type=int, default=1, help="client processes (one asyncio loop each)")
    args = ap.parse_args(argv)
    proc = None
    if args.spawn:
        port = int(args.url.rsplit(":", 1)[1])
        cmd = [sys.executable, "-m", "mlmicroservicetemplate_amd", "serve", "--model", args.spawn, "--port", str(port),
               "--host", "127.0.0.1", "--gpus", str(args.gpus), "--max-batch", str(args.max_batch), "--no-register",
               "--env-file", "/nonexistent", *args.extra.split()]
        env = dict(os.environ, PYTHONPATH=ROOT, LOG_LEVEL="warning")
        proc = subprocess.Popen(cmd, cwd=ROOT, env=env, start_new_session=True)
        if not wait_ready(args.url):
            os.killpg(proc.pid, signal.SIGKILL)
            print(json.dumps({"error": "server did not become ready"}))
            return 1
    try:
        if args.procs > 1:
            import multiprocessing as mp

            with mp.get_context("spawn").Pool(args.procs) as pool:
                parts = pool.starmap(_client_proc, [(args.url + "/predict", args.duration,
                                                     max(1, args.concurrency // args.procs), args.rate / args.procs,
                                                     args.jpeg, args.warmup, i) for i in range(args.procs)])
            lat = [x for p in parts for x in p[0]]
            errors = sum(p[1] for p in parts)
            codes = {}
            for p in parts:
                for k, v in p[2].items():
                    codes[k] = codes.get(k, 0) + v
        else:
            payloads = [make_payload(args.jpeg, s) for s in range(8)]
            lat, errors, codes = asyncio.run(run(args.url + "/predict", args.duration, args.concurrency, args.rate,
                                                 payloads, args.warmup))
    finally:
        if proc is not None:
            os.killpg(proc.pid, signal.SIGTERM)
            try:
                proc.wait(30)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
    lat_ms = np.array(lat) * 1e3 if lat else np.array([float("nan")])
    out = {
        "metric": "http requests/sec + latency", "model": args.spawn or "external", "url": args.url,
        "mode": "open" if args.rate > 0 else "closed", "concurrency": args.concurrency, "rate": args.rate,
        "payload": "jpeg" if args.jpeg else "raw-rgb8", "gpus": args.gpus, "client_procs": args.procs,
        "server_extra": args.extra,
        "requests_per_s": round(len(lat) / args.duration, 1), "p50_ms": round(float(np.percentile(lat_ms, 50)), 3),
        "p90_ms": round(float(np.percentile(lat_ms, 90)), 3), "p99_ms": round(float(np.percentile(lat_ms, 99)), 3),
        "ok": len(lat), "errors": errors, "status_codes": {str(k): v for k, v in codes.items()},
    }
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
