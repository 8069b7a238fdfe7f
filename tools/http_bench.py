"""End-to-end HTTP throughput of a serving process: starts ``python -m mlmicroservicetemplate_amd
serve`` (any model / front end / workers), waits for ``/status``, drives ``POST /predict`` with the
native closed-loop generator (``frontend/_native/mls_loadgen``) at each ``--conns`` level, and prints
one JSON line per level (requests/s, p50/p90/p99 latency, server config).

    python tools/http_bench.py --model resnet50 --frontend native --conns 64 256 --duration 10
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time

import requests

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mlmicroservicetemplate_amd.frontend import build as fbuild  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--frontend", default="native", choices=["native", "python"])
    ap.add_argument("--workers-per-gpu", type=int, default=1)
    ap.add_argument("--io-threads", type=int, default=4)
    ap.add_argument("--port", type=int, default=5099)
    ap.add_argument("--conns", type=int, nargs="+", default=[64, 256])
    ap.add_argument("--client-threads", type=int, default=4)
    ap.add_argument("--duration", type=float, default=10)
    ap.add_argument("--warmup", type=float, default=2)
    ap.add_argument("--bytes", type=int, default=224 * 224 * 3)
    ap.add_argument("--ready-timeout", type=float, default=300)
    ap.add_argument("--jpeg", action="store_true", help="upload a 320x240 JPEG (server-side decode) instead of raw RGB8")
    ap.add_argument("--decode-workers", type=int, default=4)
    ap.add_argument("--jpeg-kind", default="photo", choices=["photo", "noise"],
                    help="photo: smooth gradients + texture + mild noise (a camera-like entropy); noise: uniform "
                         "random pixels (worst case for the Huffman decoder)")
    ap.add_argument("--jpeg-size", default="320x240")
    ap.add_argument("--text", action="store_true",
                    help="upload an English text (~110 tokens) as multipart field `text` (the bert plugin)")
    args = ap.parse_args()
    fbuild.build()
    cmd = [sys.executable, "-m", "mlmicroservicetemplate_amd", "serve", "--model", args.model, "--frontend",
           args.frontend, "--port", str(args.port), "--host", "127.0.0.1", "--no-register", "--env-file", "/nonexistent",
           "--workers-per-gpu", str(args.workers_per_gpu), "--io-threads", str(args.io_threads)]
    payload_args = ["--bytes", str(args.bytes)]
    if args.jpeg:
        import io

        import numpy as np
        from PIL import Image

        buf = io.BytesIO()
        jw, jh = (int(v) for v in args.jpeg_size.split("x"))
        rng = np.random.default_rng(0)
        if args.jpeg_kind == "noise":
            img = rng.integers(0, 256, (jh, jw, 3), dtype=np.uint8)
        else:  # the fixture generator of tests/test_image_decode.py
            x = np.linspace(0, 1, jw)[None, :, None]
            y = np.linspace(0, 1, jh)[:, None, None]
            base = rng.random((1, 1, 3)) * 150 + 40 * np.sin(6 * x + rng.random() * 3) * np.cos(4 * y) + 25 * np.sin(
                18 * x * y + rng.random((1, 1, 3)))
            img = np.clip(base + rng.normal(0, 3.0, (jh, jw, 3)) + 60 * x, 0, 255).astype(np.uint8)
        Image.fromarray(img).save(buf, format="JPEG", quality=90)
        path = os.path.join(ROOT, "gpurun_out", "http_bench_upload.jpg")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "wb") as f:
            f.write(buf.getvalue())
        payload_args = ["--file", path, "--ctype", "image/jpeg"]
    if args.text:
        words = ("the quick brown fox jumps over the lazy dog while a serving framework batches "
                 "requests for the matrix cores of the accelerator").split()
        path = os.path.join(ROOT, "gpurun_out", "http_bench_upload.txt")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(" ".join(words[i % len(words)] for i in range(100)))
        payload_args = ["--file", path, "--ctype", "text/plain", "--field", "text"]
    srv = subprocess.Popen(cmd, cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT, DECODE_WORKERS=str(args.decode_workers)),
                           start_new_session=True)
    url = f"http://127.0.0.1:{args.port}"
    try:
        t0 = time.time()
        while True:
            if srv.poll() is not None:
                raise SystemExit(f"server exited with {srv.returncode}")
            try:
                r = requests.get(url + "/status", timeout=2)
                if r.status_code == 200:
                    break
                if "error" in r.json():
                    raise SystemExit(f"init failed: {r.json()}")
            except requests.RequestException:
                pass
            if time.time() - t0 > args.ready_timeout:
                raise SystemExit("server not ready")
            print(f"waiting for {url}/status ({time.time() - t0:.0f}s)", file=sys.stderr, flush=True)
            time.sleep(1)
        for conns in args.conns:
            out = subprocess.run([fbuild.loadgen_path(), "--port", str(args.port), "--conns", str(conns),
                                  "--threads", str(args.client_threads), "--duration", str(args.duration),
                                  "--warmup", str(args.warmup), *payload_args],
                                 capture_output=True, text=True, timeout=args.duration + args.warmup + 60)
            res = json.loads(out.stdout)
            try:  # server-side batching (native front end): mean samples per engine batch so far
                nat = requests.get(url + "/health", timeout=5).json().get("native") or {}
                if nat.get("batches"):
                    res["server_mean_batch"] = round(nat["samples"] / nat["batches"], 2)
                # which path tokenised / decoded the uploads (cumulative over the levels so far)
                res["server_decode_routed"] = nat.get("decode_routed")
                res["server_text_hashed"] = nat.get("text_hashed")
            except (requests.RequestException, ValueError):
                pass
            res.update({"model": args.model, "frontend": args.frontend, "workers_per_gpu": args.workers_per_gpu,
                        "io_threads": args.io_threads, "gpus": 1, "payload": "text100w" if args.text else (f"jpeg{args.jpeg_size}-{args.jpeg_kind}" if args.jpeg else "raw-rgb8"),
                        "gpu_image_decode": os.environ.get("GPU_IMAGE_DECODE", "1"),
                        "decode_workers": args.decode_workers})
            print(json.dumps(res), flush=True)
    finally:
        os.killpg(srv.pid, signal.SIGTERM)
        try:
            srv.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(srv.pid, signal.SIGKILL)
    return 0


if __name__ == "__main__":
    sys.exit(main())
