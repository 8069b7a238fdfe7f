"""API contract parity with the reference on the CPU plugins."""
import io
import os
import threading
import time
import warnings

import pytest

warnings.filterwarnings("ignore", category=DeprecationWarning)

from fastapi.testclient import TestClient  # noqa: E402
from PIL import Image  # noqa: E402

from mlmicroservicetemplate_amd.api.app import NOT_READY, READY, ROOT_MESSAGE, create_app  # noqa: E402
from mlmicroservicetemplate_amd.api.multipart import encode_multipart  # noqa: E402
from mlmicroservicetemplate_amd.config import Settings  # noqa: E402
from mlmicroservicetemplate_amd.plugins.base import ModelPlugin  # noqa: E402
from mlmicroservicetemplate_amd.plugins.builtin import IdentityPlugin, StubPlugin  # noqa: E402


def settings(**kw):
    base = {"REGISTER": False, "MAX_WAIT_US": 20000}
    base.update(kw)
    return Settings.load(env_file=None, environ={}, overrides=base)


def png_bytes():
    buf = io.BytesIO()
    Image.new("RGB", (16, 16), (0, 255, 0)).save(buf, format="PNG")
    return buf.getvalue()


def upload(data, field="image_file", filename="x.png", ctype="image/png"):
    body, ct = encode_multipart({field: (filename, data, ctype)})
    return {"content": body, "headers": {"content-type": ct}}


def wait_ready(c, timeout=5.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if c.get("/status").status_code == 200:
            return True
        time.sleep(0.01)
    return False


class GatedPlugin(StubPlugin):
    """init blocks until the test releases it."""

    def __init__(self):
        super().__init__(0)
        self.gate = threading.Event()

    def init(self, ctx):
        self.gate.wait(5)


class FailingPlugin(ModelPlugin):
    name = "failing"

    def init(self, ctx):
        raise RuntimeError("weights missing")


@pytest.fixture
def gated():
    p = GatedPlugin()
    app = create_app(settings(), p)
    with TestClient(app, raise_server_exceptions=False) as c:
        yield c, p
        p.gate.set()


def test_root_returns_list(gated):
    c, _ = gated
    r = c.get("/")
    assert r.status_code == 200
    assert r.json() == [ROOT_MESSAGE]


def test_status_transitions(gated):
    c, p = gated
    r = c.get("/status")
    assert r.status_code == 503
    assert r.json() == {"status": "failure", "detail": NOT_READY}
    p.gate.set()
    assert wait_ready(c)
    assert c.get("/status").json() == {"status": "success", "detail": READY}


def test_predict_missing_field_is_422_before_readiness(gated):
    c, _ = gated
    r = c.post("/predict")
    assert r.status_code == 422
    assert r.json()["detail"][0]["loc"] == ["body", "image_file"]
    r = c.post("/predict", **upload(png_bytes(), field="other"))
    assert r.status_code == 422


def test_predict_not_ready_503(gated):
    c, _ = gated
    r = c.post("/predict", **upload(png_bytes()))
    assert r.status_code == 503
    assert r.json() == {"status": "failure", "detail": NOT_READY}


def test_predict_stub_success_and_bad_image(gated):
    c, p = gated
    p.gate.set()
    assert wait_ready(c)
    r = c.post("/predict", **upload(png_bytes()))
    assert r.status_code == 200
    assert r.json() == {"status": "success",
                        "result": {"classes": ["isGreen", "isRed"], "result": {"isGreen": 0, "isRed": 1}}}
    r = c.post("/predict", **upload(b"definitely not an image"))
    assert r.status_code == 500


def test_malformed_multipart_is_400(gated):
    c, p = gated
    p.gate.set()
    assert wait_ready(c)
    r = c.post("/predict", content=b"--xx\r\ngarbage", headers={"content-type": "multipart/form-data; boundary=xx"})
    assert r.status_code == 400


def test_cors_allowed_origins(gated):
    c, _ = gated
    for origin in ("http://localhost", "http://localhost:3000", "http://localhost:5057", "http://localhost:5000",
                   "http://localhost:6379"):
        r = c.options("/status", headers={"Origin": origin, "Access-Control-Request-Method": "GET"})
        assert r.status_code == 200
        assert r.headers["access-control-allow-origin"] == origin
        assert r.headers["access-control-allow-credentials"] == "true"
    r = c.options("/status", headers={"Origin": "http://evil.example", "Access-Control-Request-Method": "GET"})
    assert "access-control-allow-origin" not in r.headers


def test_legacy_filename_flow(tmp_path):
    (tmp_path / "img.png").write_bytes(png_bytes())
    app = create_app(settings(IMAGE_DIR=str(tmp_path)), StubPlugin(0))
    with TestClient(app, raise_server_exceptions=False) as c:
        assert wait_ready(c)
        r = c.post("/predict?filename=img.png")
        assert r.status_code == 200 and r.json()["status"] == "success"
        r = c.post("/predict?filename=nope.png")
        assert r.status_code == 400
        assert r.json() == {"status": "failure",
                            "detail": "Invalid file name provided: [nope.png]. Unable to find image on server."}
        r = c.post("/predict?filename=../../etc/passwd")
        assert r.status_code == 400


def test_init_failure_reported():
    app = create_app(settings(), FailingPlugin())
    with TestClient(app, raise_server_exceptions=False) as c:
        t0 = time.time()
        while time.time() - t0 < 5:
            r = c.get("/status")
            if "error" in r.json():
                break
            time.sleep(0.01)
        assert r.status_code == 503
        assert "weights missing" in r.json()["error"]
        assert c.get("/health").json()["init_error"].startswith("RuntimeError")


def test_identity_batches_concurrent_requests():
    app = create_app(settings(MAX_BATCH=8, MAX_WAIT_US=50000), IdentityPlugin())
    import zlib
    from concurrent.futures import ThreadPoolExecutor

    with TestClient(app, raise_server_exceptions=False) as c:
        assert wait_ready(c)
        payloads = [os.urandom(100 + i) for i in range(16)]

        def call(p):
            return c.post("/predict", **upload(p, ctype="application/octet-stream")).json()

        with ThreadPoolExecutor(16) as ex:
            outs = list(ex.map(call, payloads))
        for p, o in zip(payloads, outs):
            assert o["status"] == "success"
            assert o["result"]["result"] == {"bytes": len(p), "crc32": zlib.crc32(p) & 0xFFFFFFFF}
        assert max(o["result"]["batch_size"] for o in outs) > 1
        m = c.get("/metrics").text
        assert "mlsamd_batch_size_bucket" in m
        assert 'mlsamd_requests_total{route="/predict",status="200"} 16.0' in m


def test_generate_on_non_llm(gated):
    c, p = gated
    p.gate.set()
    assert wait_ready(c)
    assert c.post("/generate", json={"prompt": "hi"}).status_code == 400
    assert c.post("/generate", json={"nothing": 1}).status_code == 422


def test_module_plugin_reference_contract(tmp_path, monkeypatch):
    mod = tmp_path / "my_model.py"
    mod.write_text(
        "CALLS = []\n"
        "def init():\n    CALLS.append('init')\n"
        "def predict(image_file):\n    return {'n': len(image_file.file.read()), 'name': image_file.filename}\n"
    )
    monkeypatch.syspath_prepend(str(tmp_path))
    app = create_app(settings(MODEL="my_model"))
    with TestClient(app, raise_server_exceptions=False) as c:
        assert wait_ready(c)
        r = c.post("/predict", **upload(b"12345", filename="f.bin"))
        assert r.json() == {"status": "success", "result": {"n": 5, "name": "f.bin"}}


def test_urlencoded_text_field():
    """A url-encoded form carrying the plugin's field is a prediction input (text plugins)."""
    import zlib

    app = create_app(settings(), IdentityPlugin())
    with TestClient(app, raise_server_exceptions=False) as c:
        assert wait_ready(c)
        r = c.post("/predict", content=b"image_file=hello+world&x=1",
                   headers={"content-type": "application/x-www-form-urlencoded"})
        assert r.status_code == 200, r.text
        assert r.json()["result"]["result"]["crc32"] == zlib.crc32(b"hello world") & 0xFFFFFFFF


def test_request_timeout_is_504():
    import threading

    from mlmicroservicetemplate_amd.plugins.base import ModelPlugin

    release = threading.Event()

    class Slow(ModelPlugin):
        name = "slow"
        batched = True

        def preprocess(self, part):
            return part.data

        def replicas(self):
            def run_batch(samples):
                release.wait(5)
                return [{"n": len(x)} for x in samples]
            return [run_batch]

        def postprocess(self, out):
            return out

    app = create_app(settings(REQUEST_TIMEOUT_S=0.2, WATCHDOG_INTERVAL_S=0), Slow())
    with TestClient(app, raise_server_exceptions=False) as c:
        assert wait_ready(c)
        r = c.post("/predict", **upload(b"abc", ctype="application/octet-stream"))
        assert r.status_code == 504 and r.json()["detail"] == "Prediction timed out."
        release.set()



def test_upload_limit_applies_to_every_body_type():
    """MAX_UPLOAD_BYTES -> 413 for multipart, JSON and urlencoded /predict bodies and for
    /generate and /admin/reload JSON, by Content-Length and by streamed (chunked) length."""
    with TestClient(create_app(settings(MAX_UPLOAD_BYTES=1000, API_KEY="k"), IdentityPlugin())) as c:
        assert wait_ready(c)
        big = b"x" * 2000
        too_large = {"status": "failure", "detail": "Upload too large."}
        for kw in (upload(big),
                   {"content": b'{"image_file": "' + big + b'"}', "headers": {"content-type": "application/json"}},
                   {"content": b"image_file=" + big, "headers": {"content-type": "application/x-www-form-urlencoded"}}):
            r = c.post("/predict", **kw)
            assert r.status_code == 413 and r.json() == too_large
        for path in ("/generate", "/admin/reload"):
            r = c.post(path, content=b'{"prompt": "' + big + b'"}',
                       headers={"content-type": "application/json", "api_key": "k"})
            assert r.status_code == 413 and r.json() == too_large

        def chunks():  # no Content-Length: the streamed length is checked
            for _ in range(4):
                yield b"x" * 400

        r = c.post("/predict", content=chunks(), headers={"content-type": "application/json"})
        assert r.status_code == 413
        assert c.post("/predict", **upload(b"y" * 100)).status_code == 200
