"""Native C++ front end (FRONTEND=native, frontend/csrc/httpfront.cpp) on CPU: wire parity with
the reference contract and the FastAPI app, C++ micro-batching, decode / legacy / admission
paths, the C++ load generator, and the launcher.  Uses the CPU ``toy_classifier`` plugin."""
import io
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
import warnings

import numpy as np
import pytest
import requests

warnings.filterwarnings("ignore", category=DeprecationWarning)

from fastapi.testclient import TestClient  # noqa: E402
from PIL import Image  # noqa: E402

from mlmicroservicetemplate_amd.api.app import create_app  # noqa: E402
from mlmicroservicetemplate_amd.api.multipart import encode_multipart  # noqa: E402
from mlmicroservicetemplate_amd.config import Settings  # noqa: E402
from mlmicroservicetemplate_amd.frontend import build as fbuild  # noqa: E402
from mlmicroservicetemplate_amd.frontend.native import HostReplica, NativeService, load_extension  # noqa: E402
from mlmicroservicetemplate_amd.plugins.base import PluginContext  # noqa: E402
from mlmicroservicetemplate_amd.plugins.builtin import ToyClassifierPlugin  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NOT_READY = {"status": "failure", "detail": "Model is not ready to receive predictions."}


def settings(**kw):
    base = {"MODEL": "toy_classifier", "REGISTER": False, "MAX_WAIT_US": 5000, "IO_THREADS": 2}
    base.update(kw)
    return Settings.load(env_file=None, environ={}, overrides=base)


def img(seed=0, size=8):
    return np.random.default_rng(seed).integers(0, 256, (size, size, 3), dtype=np.uint8)


def raw_upload(a, field="image_file"):
    body, ct = encode_multipart({field: ("x.rgb", a.tobytes(), "application/octet-stream")})
    return {"data": body, "headers": {"content-type": ct}}


@pytest.fixture(scope="module", autouse=True)
def _ext():
    load_extension()  # builds in-tree if needed; fails loudly otherwise


class Service:
    def __init__(self, plugin=None, auto_init=True, **kw):
        self.s = settings(**kw)
        self.plugin = plugin or ToyClassifierPlugin()
        self.svc = NativeService(self.s, self.plugin, PluginContext(settings=self.s), host="127.0.0.1", port=0)
        self.svc.start(auto_init=auto_init)
        self.url = f"http://127.0.0.1:{self.svc.port}"

    def wait_ready(self, timeout=5.0):
        t0 = time.time()
        while time.time() - t0 < timeout:
            if requests.get(self.url + "/status", timeout=2).status_code == 200:
                return True
            time.sleep(0.01)
        return False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.svc.stop()


def test_routes_and_prediction_match_model():
    with Service() as s:
        r = requests.get(s.url + "/", timeout=5)
        assert r.status_code == 200 and r.json() == ["MLMicroserviceTemplate is Running!"]
        assert s.wait_ready()
        assert requests.get(s.url + "/status").json() == {
            "status": "success", "detail": "Model ready to receive prediction requests."}
        a = img(1)
        r = requests.post(s.url + "/predict", **raw_upload(a), timeout=5)
        assert r.status_code == 200, r.text
        body = r.json()
        assert body["status"] == "success"
        vals, idx = s.plugin.scores(a[None])
        names = [f"class_{i}" for i in idx[0]]
        assert body["result"]["classes"] == names
        got = [body["result"]["result"][n] for n in names]
        np.testing.assert_allclose(got, vals[0], rtol=1e-6)
        # whole-body octet-stream upload takes the same path
        r = requests.post(s.url + "/predict", data=a.tobytes(), headers={"content-type": "application/octet-stream"})
        assert r.status_code == 200 and r.json() == body


def test_parity_with_python_frontend():
    """Same plugin, same request -> same result through FastAPI and through the C++ front end."""
    a = img(7)
    plugin = ToyClassifierPlugin()
    with TestClient(create_app(settings(), plugin)) as c:
        for _ in range(200):
            if c.get("/status").status_code == 200:
                break
            time.sleep(0.01)
        up = raw_upload(a)
        py = c.post("/predict", content=up["data"], headers=up["headers"]).json()
        py_missing = c.post("/predict", content=b"", headers={"content-type": "multipart/form-data; boundary=b"})
    with Service() as s:
        assert s.wait_ready()
        nat = requests.post(s.url + "/predict", **raw_upload(a)).json()
        nat_missing = requests.post(s.url + "/predict", data=b"--b--\r\n",
                                    headers={"content-type": "multipart/form-data; boundary=b"})
    assert nat["result"]["classes"] == py["result"]["classes"]
    for k, v in py["result"]["result"].items():
        assert abs(nat["result"]["result"][k] - v) < 1e-6
    assert nat_missing.status_code == 422 and nat_missing.json() == {
        "detail": [{"type": "missing", "loc": ["body", "image_file"], "msg": "Field required", "input": None}]}
    assert py_missing.status_code in (400, 422)


def test_not_ready_then_ready_and_validation_order():
    with Service(auto_init=False) as s:
        r = requests.get(s.url + "/status")
        assert r.status_code == 503 and r.json() == NOT_READY
        # missing field -> 422 even before readiness (FastAPI validation runs first, main.py:119-131)
        r = requests.post(s.url + "/predict")
        assert r.status_code == 422
        r = requests.post(s.url + "/predict", **raw_upload(img()))
        assert r.status_code == 503 and r.json() == NOT_READY
        s.svc._init()
        assert requests.get(s.url + "/status").status_code == 200
        assert requests.post(s.url + "/predict", **raw_upload(img())).status_code == 200


class BrokenToy(ToyClassifierPlugin):
    def init(self, ctx):
        raise RuntimeError("weights missing")


def test_init_failure_reported():
    with Service(plugin=BrokenToy()) as s:
        t0 = time.time()
        while time.time() - t0 < 5:
            r = requests.get(s.url + "/status")
            if "error" in r.json():
                break
            time.sleep(0.02)
        assert r.status_code == 503
        assert "weights missing" in r.json()["error"]


def test_errors_404_405_malformed_and_health_metrics():
    with Service() as s:
        assert s.wait_ready()
        r = requests.get(s.url + "/nope")
        assert r.status_code == 404 and r.json() == {"detail": "Not Found"}
        r = requests.get(s.url + "/predict")
        assert r.status_code == 405 and r.headers["allow"] == "POST"
        r = requests.post(s.url + "/predict", data=b"garbage", headers={"content-type": "multipart/form-data; boundary=zz"})
        assert r.status_code == 400
        h = requests.get(s.url + "/health").json()
        assert h["ready"] and h["frontend"] == "native" and h["replicas"][0]["healthy"]
        m = requests.get(s.url + "/metrics")
        assert m.status_code == 200 and "mls_native_requests_total" in m.text and 'code="404"' in m.text
        info = requests.get(s.url + "/info").json()
        assert info["frontend"] == "native" and info["settings"]["MODEL"] == "toy_classifier"


def test_decode_path_and_bad_image():
    a = img(3)
    buf = io.BytesIO()
    Image.fromarray(a).save(buf, format="PNG")
    with Service() as s:
        assert s.wait_ready()
        raw = requests.post(s.url + "/predict", **raw_upload(a)).json()
        body, ct = encode_multipart({"image_file": ("x.png", buf.getvalue(), "image/png")})
        png = requests.post(s.url + "/predict", data=body, headers={"content-type": ct})
        assert png.status_code == 200 and png.json() == raw  # lossless PNG decodes to the same pixels
        body, ct = encode_multipart({"image_file": ("x.txt", b"not an image", "text/plain")})
        r = requests.post(s.url + "/predict", data=body, headers={"content-type": ct})
        assert r.status_code == 500  # PIL cannot identify it (reference model.py:23 -> 500)
        assert s.svc.srv.stats()["decode_routed"] == 2


def test_cors_allowed_and_preflight():
    with Service() as s:
        r = requests.get(s.url + "/", headers={"Origin": "http://localhost:3000"})
        assert r.headers["access-control-allow-origin"] == "http://localhost:3000"
        assert r.headers["access-control-allow-credentials"] == "true"
        r = requests.get(s.url + "/", headers={"Origin": "http://evil.example"})
        assert "access-control-allow-origin" not in r.headers
        r = requests.options(s.url + "/predict", headers={"Origin": "http://localhost:5000",
                                                          "Access-Control-Request-Method": "POST",
                                                          "Access-Control-Request-Headers": "content-type"})
        assert r.status_code == 200 and r.headers["access-control-allow-origin"] == "http://localhost:5000"
        assert "POST" in r.headers["access-control-allow-methods"]
        r = requests.options(s.url + "/predict", headers={"Origin": "http://evil.example",
                                                          "Access-Control-Request-Method": "POST"})
        assert r.status_code == 400


def test_concurrent_requests_are_batched():
    with Service(MAX_WAIT_US=20000) as s:
        assert s.wait_ready()
        results = {}

        def one(i):
            with requests.Session() as sess:
                r = sess.post(s.url + "/predict", **raw_upload(img(i)), timeout=10)
                results[i] = r

        ths = [threading.Thread(target=one, args=(i,)) for i in range(48)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert all(r.status_code == 200 for r in results.values())
        for i, r in results.items():  # each response belongs to its own request
            _, idx = s.plugin.scores(img(i)[None])
            assert r.json()["result"]["classes"] == [f"class_{k}" for k in idx[0]]
        st = s.svc.srv.stats()
        assert st["samples"] == 48 and st["batches"] < 48


def _recv_responses(sock, n, timeout=5.0):
    sock.settimeout(timeout)
    buf = b""
    out = []
    while len(out) < n:
        while b"\r\n\r\n" not in buf:
            buf += sock.recv(65536)
        head, rest = buf.split(b"\r\n\r\n", 1)
        clen = int([ln.split(b":")[1] for ln in head.split(b"\r\n") if ln.lower().startswith(b"content-length")][0])
        while len(rest) < clen:
            rest += sock.recv(65536)
        out.append((int(head.split(b" ")[1]), rest[:clen]))
        buf = rest[clen:]
    return out


def test_keepalive_pipelining_in_order():
    with Service() as s:
        assert s.wait_ready()
        up = raw_upload(img(5))
        req = (b"POST /predict HTTP/1.1\r\nHost: x\r\nContent-Type: " + up["headers"]["content-type"].encode() +
               b"\r\nContent-Length: " + str(len(up["data"])).encode() + b"\r\n\r\n" + up["data"])
        with socket.create_connection(("127.0.0.1", s.svc.port)) as sock:
            sock.sendall(b"GET / HTTP/1.1\r\nHost: x\r\n\r\n" + req + b"GET /nope HTTP/1.1\r\nHost: x\r\n\r\n" + req)
            got = _recv_responses(sock, 4)
        assert [c for c, _ in got] == [200, 200, 404, 200]
        assert json.loads(got[0][1]) == ["MLMicroserviceTemplate is Running!"]
        assert json.loads(got[1][1]) == json.loads(got[3][1])


class SlowToy(ToyClassifierPlugin):
    def native_replicas(self):
        def fn(x):
            time.sleep(0.3)
            return self.scores(x)

        return [HostReplica(fn, (8, 8, 3), 1, 1)]


def test_admission_control_and_timeout():
    with Service(plugin=SlowToy(), MAX_QUEUE=2, MAX_BATCH=1, MAX_WAIT_US=0) as s:
        assert s.wait_ready()
        codes = []
        lock = threading.Lock()

        def one(i):
            r = requests.post(s.url + "/predict", **raw_upload(img(i)), timeout=20)
            with lock:
                codes.append((r.status_code, r.headers.get("retry-after")))

        ths = [threading.Thread(target=one, args=(i,)) for i in range(8)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert any(c == 200 for c, _ in codes)
        assert any(c == 503 and ra == "1" for c, ra in codes)
    with Service(plugin=SlowToy(), MAX_BATCH=1, MAX_WAIT_US=0, REQUEST_TIMEOUT_S=0.1) as s:
        assert s.wait_ready()
        out = []
        ths = [threading.Thread(target=lambda i=i: out.append(
            requests.post(s.url + "/predict", **raw_upload(img(i)), timeout=20).status_code)) for i in range(4)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert 504 in out and 200 in out


def test_legacy_filename_flow(tmp_path):
    a = img(9)
    Image.fromarray(a).save(tmp_path / "x.png")
    with Service(IMAGE_DIR=str(tmp_path)) as s:
        assert s.wait_ready()
        ok = requests.post(s.url + "/predict?filename=x.png")
        assert ok.status_code == 200
        assert ok.json() == requests.post(s.url + "/predict", **raw_upload(a)).json()
        bad = requests.post(s.url + "/predict?filename=missing.png")
        assert bad.status_code == 400 and "Invalid file name provided: [missing.png]" in bad.json()["detail"]
        esc = requests.post(s.url + "/predict", json={"filename": "../../etc/passwd"})
        assert esc.status_code == 400


def test_native_loadgen_binary():
    with Service(MAX_WAIT_US=1000) as s:
        assert s.wait_ready()
        out = subprocess.run([fbuild.loadgen_path(), "--port", str(s.svc.port), "--conns", "8", "--threads", "2",
                              "--duration", "1", "--warmup", "0.2", "--bytes", "192"],
                             capture_output=True, text=True, timeout=30)
        res = json.loads(out.stdout)
        assert res["ok"] > 100 and res["errors"] == 0 and res["status_codes"] == {"200": res["ok"]}
        assert res["p50_ms"] > 0


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


@pytest.mark.timeout(90)
def test_launcher_serves_native_and_stops_on_sigterm():
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    proc = subprocess.Popen([sys.executable, "-m", "mlmicroservicetemplate_amd", "serve", "--model", "toy_classifier",
                             "--frontend", "native", "--port", str(port), "--host", "127.0.0.1", "--no-register",
                             "--env-file", "/nonexistent"], cwd=ROOT, env=env, start_new_session=True)
    try:
        url = f"http://127.0.0.1:{port}"
        deadline = time.time() + 60
        ready = False
        while time.time() < deadline and not ready:
            try:
                ready = requests.get(url + "/status", timeout=1).status_code == 200
            except requests.RequestException:
                time.sleep(0.2)
        assert ready
        r = requests.post(url + "/predict", **raw_upload(img(2)))
        assert r.status_code == 200 and r.headers["server"] == "mls-native"
        proc.send_signal(signal.SIGTERM)
        assert proc.wait(30) == 0
    finally:
        if proc.poll() is None:
            os.killpg(proc.pid, signal.SIGKILL)


@pytest.mark.timeout(120)
def test_two_rank_native_service_shares_the_port():
    """GPUS=2 (gloo on CPU): two ranks, each a native front end on the launcher's shared listening
    socket (EPOLLEXCLUSIVE accept across processes)."""
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    proc = subprocess.Popen([sys.executable, "-m", "mlmicroservicetemplate_amd", "serve", "--model", "toy_classifier",
                             "--frontend", "native", "--gpus", "2", "--port", str(port), "--host", "127.0.0.1",
                             "--no-register", "--env-file", "/nonexistent"], cwd=ROOT, env=env, start_new_session=True)
    try:
        url = f"http://127.0.0.1:{port}"
        deadline = time.time() + 90
        ready = False
        while time.time() < deadline and not ready:
            try:
                ready = requests.get(url + "/status", timeout=1).status_code == 200
            except requests.RequestException:
                time.sleep(0.2)
        assert ready
        ranks = set()
        for i in range(200):
            info = requests.get(url + "/info", timeout=5).json()  # new connection each time
            assert info["world_size"] == 2
            r = requests.post(url + "/predict", **raw_upload(img(i)), timeout=5)
            if r.status_code == 503:  # /status answered from a ready rank; this one is still loading
                time.sleep(0.1)
                continue
            assert r.status_code == 200
            ranks.add(info["rank"])
            if len(ranks) == 2:
                break
        assert ranks == {0, 1}
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)


def _raw_exchange(port, data, timeout=5.0):
    with socket.create_connection(("127.0.0.1", port), timeout=timeout) as sk:
        sk.sendall(data)
        sk.shutdown(socket.SHUT_WR)
        buf = b""
        while True:
            chunk = sk.recv(65536)
            if not chunk:
                break
            buf += chunk
    return buf


def test_http_protocol_edges():
    """HTTP/1.0 close, Expect: 100-continue, chunked -> 411, oversize -> 413, huge header -> 431,
    bad Content-Length / request line -> 400."""
    with Service(MAX_UPLOAD_BYTES=4096) as s:
        assert s.wait_ready()
        port = s.svc.port
        r = _raw_exchange(port, b"GET / HTTP/1.0\r\n\r\n")
        assert r.startswith(b"HTTP/1.1 200") and b"connection: close" in r.lower()
        up = raw_upload(img(1))
        head = (b"POST /predict HTTP/1.1\r\nHost: x\r\nExpect: 100-continue\r\nContent-Type: " +
                up["headers"]["content-type"].encode() + b"\r\nContent-Length: " + str(len(up["data"])).encode() +
                b"\r\n\r\n")
        with socket.create_connection(("127.0.0.1", port), timeout=5) as sk:
            sk.sendall(head)
            first = sk.recv(1024)
            assert first.startswith(b"HTTP/1.1 100 Continue")
            sk.sendall(up["data"])
            got = _recv_responses(sk, 1)
            assert got[0][0] == 200
        r = _raw_exchange(port, b"POST /predict HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n0\r\n\r\n")
        assert r.startswith(b"HTTP/1.1 411")
        r = _raw_exchange(port, b"POST /predict HTTP/1.1\r\nContent-Length: 999999\r\n\r\n")
        assert r.startswith(b"HTTP/1.1 413")
        r = _raw_exchange(port, b"GET / HTTP/1.1\r\nX-Big: " + b"a" * 70000 + b"\r\n\r\n")
        assert r.startswith(b"HTTP/1.1 431")
        r = _raw_exchange(port, b"POST /predict HTTP/1.1\r\nContent-Length: 12x\r\n\r\n")
        assert r.startswith(b"HTTP/1.1 400")
        r = _raw_exchange(port, b"GARBAGE\r\n\r\n")
        assert r.startswith(b"HTTP/1.1 400")
        # the server is still healthy after the abuse
        assert requests.post(s.url + "/predict", **raw_upload(img(2))).status_code == 200
