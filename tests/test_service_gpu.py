"""The whole serving stack on MI355X (in-process ASGI): HTTP multipart -> decode -> dynamic
batcher -> GPU engine (concurrent slots, hipGraphs of the fused kernels) -> JSON, for the
ResNet-50 (config 2), BERT (config 3) and Llama /generate (config 5, tiny shapes) plugins, checked
against the same models called directly."""
import io
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _client(**over):
    from fastapi.testclient import TestClient

    from mlmicroservicetemplate_amd.api.app import create_app
    from mlmicroservicetemplate_amd.config import Settings

    base = {"REGISTER": False, "GPUS": 1, "MAX_WAIT_US": 20000, "WATCHDOG_STALL_S": 120}
    base.update(over)
    return TestClient(create_app(Settings.load(env_file=None, environ={}, overrides=base)),
                      raise_server_exceptions=False)


def _wait(c, timeout=300):
    t0 = time.time()
    while time.time() - t0 < timeout:
        r = c.get("/status")
        if r.status_code == 200:
            return
        assert "error" not in r.json(), r.json()
        time.sleep(0.1)
    raise AssertionError("service not ready")


def _png(seed, size=(300, 260)):
    from PIL import Image

    rng = np.random.default_rng(seed)
    img = Image.fromarray(rng.integers(0, 256, (size[1], size[0], 3), dtype=np.uint8))
    buf = io.BytesIO()
    img.save(buf, format="PNG")
    return buf.getvalue()


def test_resnet50_service_matches_direct_model():
    from mlmicroservicetemplate_amd.models import resnet
    from mlmicroservicetemplate_amd.plugins.builtin import decode_image

    with _client(MODEL="resnet50", MAX_BATCH=8, GRAPH_BUCKETS=[1, 2, 4, 8]) as c:
        _wait(c)
        imgs = [_png(i) for i in range(12)]
        with ThreadPoolExecutor(12) as ex:
            outs = list(ex.map(lambda b: c.post("/predict", files={"image_file": ("x.png", b, "image/png")}), imgs))
        assert all(o.status_code == 200 for o in outs), [o.text for o in outs if o.status_code != 200]
        res = [o.json()["result"] for o in outs]
        assert all(len(r["classes"]) == 5 for r in res)
        # the same images through the model directly (same seed-0 weights, fp32 reference)
        x = torch.from_numpy(np.stack([decode_image(b, "image/png") for b in imgs])).cuda()
        ref = resnet.resnet50_reference({k: v.cuda() for k, v in resnet.init_resnet50(0).items()}, x).float()
        got = torch.tensor([int(r["classes"][0].split("_")[1]) for r in res], device=ref.device)
        # margin rule: exact top-1 on every image whose reference top-2 gap exceeds 1e-2 of the
        # largest logit (a near-tie may flip under bf16 rounding and batch-bucket tile choices)
        top2 = ref.topk(2, dim=-1).values
        sure = (top2[:, 0] - top2[:, 1]) / ref.abs().max() > 1e-2
        assert sure.sum() >= len(imgs) // 2, "too few decisive images to test anything"
        assert torch.equal(got[sure], ref.argmax(-1)[sure]), (got, ref.argmax(-1), sure)
        h = c.get("/health").json()
        assert h["replicas"][0]["healthy"] and h["replicas"][0]["batches"] >= 2
        assert c.get("/info").json()["model"]["engines"][0]["concurrent"]


def test_bert_service():
    with _client(MODEL="bert", MAX_BATCH=8, GRAPH_BUCKETS=[1, 2, 4, 8]) as c:
        _wait(c)
        texts = ["the quick brown fox", "MI355X serving " * 20, "a"]
        with ThreadPoolExecutor(3) as ex:
            outs = list(ex.map(lambda t: c.post("/predict", data={"text": t}), texts))
        assert all(o.status_code == 200 for o in outs), [o.text for o in outs]
        assert all(len(o.json()["result"]["classes"]) >= 1 for o in outs)


def test_llama_generate_service_fused(tmp_path):
    from mlmicroservicetemplate_amd.models.llama import GenParams, LlamaTP, init_llama_shard, tiny_config

    y = tmp_path / "llama.yaml"
    y.write_text("config: tiny\nmax_seq: 256\noverrides:\n  layers: 2\n  head_dim: 128\n  heads: 4\n  kv_heads: 1\n")
    with _client(MODEL="llama", MODEL_CONFIG=str(y), MAX_BATCH=4, BACKEND="fused") as c:
        _wait(c)
        ids = [1, 55, 99, 1000, 7, 8]
        r = c.post("/generate", json={"input_ids": ids, "max_new_tokens": 6})
        assert r.status_code == 200, r.text
        res = r.json()["result"]
        cfg = tiny_config(layers=2, head_dim=128, heads=4, kv_heads=1)
        m = LlamaTP(init_llama_shard(cfg, 1, 0, seed=0, device="cuda"), cfg, backend="fused", device="cuda",
                    max_batch=4, max_seq=256)
        want = m.generate(torch.tensor([ids], device="cuda"), torch.tensor([len(ids)], device="cuda"),
                          GenParams(6))[0].tolist()
        assert res["token_ids"] == want[: res["num_tokens"]]


def test_resnet50_native_frontend_matches_python_frontend():
    """FRONTEND=native: C++ HTTP + C++ batcher writing straight into the engine slot's pinned
    buffer -> same top-5 as the FastAPI path for raw and PNG uploads, and the C++ load generator
    drives it without errors."""
    import json
    import subprocess

    import requests

    from mlmicroservicetemplate_amd.api.multipart import encode_multipart
    from mlmicroservicetemplate_amd.config import Settings
    from mlmicroservicetemplate_amd.frontend import build as fbuild
    from mlmicroservicetemplate_amd.frontend.native import NativeService
    from mlmicroservicetemplate_amd.plugins.base import PluginContext
    from mlmicroservicetemplate_amd.plugins.builtin import ResNet50Plugin

    rng = np.random.default_rng(0)
    raws = [rng.integers(0, 256, (224, 224, 3), dtype=np.uint8) for _ in range(6)]
    pngs = [_png(i) for i in range(3)]

    def ups():
        out = []
        for a in raws:
            out.append(encode_multipart({"image_file": ("x.rgb", a.tobytes(), "application/octet-stream")}))
        for b in pngs:
            out.append(encode_multipart({"image_file": ("x.png", b, "image/png")}))
        return out

    with _client(MODEL="resnet50", MAX_BATCH=8, GRAPH_BUCKETS=[1, 2, 4, 8]) as c:
        _wait(c)
        py = [c.post("/predict", content=b, headers={"content-type": ct}).json()["result"] for b, ct in ups()]
    s = Settings.load(env_file=None, environ={}, overrides={"REGISTER": False, "GPUS": 1, "MODEL": "resnet50",
                                                            "MAX_BATCH": 8, "GRAPH_BUCKETS": [1, 2, 4, 8],
                                                            "MAX_WAIT_US": 2000, "IO_THREADS": 2})
    svc = NativeService(s, ResNet50Plugin(), PluginContext(settings=s, devices=["cuda:0"]), host="127.0.0.1", port=0)
    svc.start()
    try:
        url = f"http://127.0.0.1:{svc.port}"
        t0 = time.time()
        while requests.get(url + "/status").status_code != 200:
            assert time.time() - t0 < 300 and "error" not in requests.get(url + "/status").json()
            time.sleep(0.1)
        # one at a time: both front ends run each image as a batch of 1 (same bucket graph) -> same bits
        outs = [requests.post(url + "/predict", data=b, headers={"content-type": ct}, timeout=60) for b, ct in ups()]
        assert all(o.status_code == 200 for o in outs), [o.text for o in outs]
        nat = [o.json()["result"] for o in outs]
        for a, b in zip(py, nat):
            assert a["classes"] == b["classes"]
            for k in a["result"]:
                assert abs(a["result"][k] - b["result"][k]) < 1e-5
        # concurrently: micro-batched into larger buckets (other tile plans, bf16 rounding differs)
        with ThreadPoolExecutor(9) as ex:
            outs = list(ex.map(lambda u: requests.post(url + "/predict", data=u[0], headers={"content-type": u[1]},
                                                       timeout=60), ups()))
        assert all(o.status_code == 200 for o in outs), [o.text for o in outs]
        # margin rule against the fp32 reference of the same uploads (decoded as the service does)
        from mlmicroservicetemplate_amd.models import resnet
        from mlmicroservicetemplate_amd.plugins.builtin import decode_image

        x = torch.from_numpy(np.stack([a for a in raws] + [decode_image(b, "image/png") for b in pngs])).cuda()
        ref = resnet.resnet50_reference({k: v.cuda() for k, v in resnet.init_resnet50(0).items()}, x).float()
        top2 = ref.topk(2, dim=-1).values
        sure = ((top2[:, 0] - top2[:, 1]) / ref.abs().max() > 1e-2).tolist()
        want = ref.argmax(-1).tolist()
        assert sum(sure) >= 4, "too few decisive images to test anything"
        for i, o in enumerate(outs):
            cls = int(o.json()["result"]["classes"][0].split("_")[1])
            if sure[i]:
                assert cls == want[i], (i, cls, want[i])
        lg = subprocess.run([fbuild.loadgen_path(), "--port", str(svc.port), "--conns", "32", "--threads", "2",
                             "--duration", "2", "--warmup", "0.5"], capture_output=True, text=True, timeout=60)
        res = json.loads(lg.stdout)
        assert res["errors"] == 0 and res["ok"] > 100, res
        st = svc.srv.stats()
        assert st["samples"] > st["batches"]  # requests were micro-batched
    finally:
        svc.stop()


def test_bert_native_frontend_matches_python_frontend():
    """FRONTEND=native with the bert plugin (config 3): the Python decode thread tokenises straight
    into the engine's packed row, the C++ batcher packs rows into the slot's pinned buffer; the
    top class matches the FastAPI path (which may pick a shorter seq bucket: probabilities within
    bf16 noise) for multipart, JSON and urlencoded texts, and a same-size text body is never taken
    as a raw row."""
    import json
    import subprocess

    import requests

    from mlmicroservicetemplate_amd.config import Settings
    from mlmicroservicetemplate_amd.frontend import build as fbuild
    from mlmicroservicetemplate_amd.frontend.native import NativeService
    from mlmicroservicetemplate_amd.plugins.base import PluginContext
    from mlmicroservicetemplate_amd.plugins.text_classifier import BertPlugin

    texts = ["the quick brown fox", "MI355X serving " * 20, "a", "x" * ((2 * 128 + 1) * 4)]
    with _client(MODEL="bert", MAX_BATCH=8, GRAPH_BUCKETS=[1, 2, 4, 8]) as c:
        _wait(c)
        py = [c.post("/predict", data={"text": t}).json()["result"] for t in texts]
    s = Settings.load(env_file=None, environ={}, overrides={"REGISTER": False, "GPUS": 1, "MODEL": "bert",
                                                            "MAX_BATCH": 8, "GRAPH_BUCKETS": [1, 2, 4, 8],
                                                            "MAX_WAIT_US": 2000, "IO_THREADS": 2})
    svc = NativeService(s, BertPlugin(), PluginContext(settings=s, devices=["cuda:0"]), host="127.0.0.1", port=0)
    svc.start()
    try:
        url = f"http://127.0.0.1:{svc.port}"
        t0 = time.time()
        while requests.get(url + "/status").status_code != 200:
            assert time.time() - t0 < 300 and "error" not in requests.get(url + "/status").json()
            time.sleep(0.1)
        outs = [requests.post(url + "/predict", files={"text": (None, t)}, timeout=60) for t in texts]
        outs += [requests.post(url + "/predict", json={"text": texts[0]}, timeout=60),
                 requests.post(url + "/predict", data={"text": texts[1]}, timeout=60)]
        assert all(o.status_code == 200 for o in outs), [o.text for o in outs]
        nat = [o.json()["result"] for o in outs]
        for a, b in zip(py + [py[0], py[1]], nat):
            assert a["classes"][0] == b["classes"][0]
            for k in a["result"]:
                assert abs(a["result"][k] - b["result"][k]) < 2e-2
        lg = subprocess.run([fbuild.loadgen_path(), "--port", str(svc.port), "--conns", "32", "--threads", "2",
                             "--duration", "2", "--warmup", "0.5", "--field", "text", "--bytes", "400"],
                            capture_output=True, text=True, timeout=60)
        res = json.loads(lg.stdout)
        assert res["errors"] == 0 and res["ok"] > 100, res
        st = svc.srv.stats()
        assert st["samples"] > st["batches"]  # requests were micro-batched
    finally:
        svc.stop()


def test_resnet50_hot_reload_in_place_under_graphs():
    """POST /admin/reload's engine path: new weights copied INTO the tensors the captured hipGraphs
    read (pointers unchanged, no re-capture), outputs equal a model built from the new weights."""
    from mlmicroservicetemplate_amd.config import Settings
    from mlmicroservicetemplate_amd.models import resnet
    from mlmicroservicetemplate_amd.ops import autotune
    from mlmicroservicetemplate_amd.plugins.base import PluginContext
    from mlmicroservicetemplate_amd.plugins.builtin import ResNet50Plugin

    s = Settings.load(env_file=None, environ={}, overrides={"REGISTER": False, "GPUS": 1, "MODEL": "resnet50",
                                                            "MAX_BATCH": 4, "GRAPH_BUCKETS": [4], "INFLIGHT": 2})
    plugin = ResNet50Plugin()
    plugin.init(PluginContext(settings=s, devices=["cuda:0"]))
    from mlmicroservicetemplate_amd.plugins.builtin import image_container

    eng, model = plugin.engines[0], plugin.models[0]
    x = np.random.default_rng(3).integers(0, 256, (4, 224, 224, 3), dtype=np.uint8)
    assert plugin.containers  # engine rows are GPU image containers (raw uploads wrapped)
    xc = np.stack([image_container(img.tobytes(), "application/octet-stream") for img in x])
    v0, i0 = eng.run(xc)
    ptrs = {k: t.data_ptr() for k, t in model.w.items()}
    params1 = plugin.load_params(None, 1)
    plugin.apply_params(params1)
    assert {k: t.data_ptr() for k, t in model.w.items()} == ptrs
    v1, i1 = eng.run(xc)  # graph replay on the reloaded weights
    fresh = resnet.ResNet50Fused(params1, "cuda:0", max_batch=4, tuning=autotune.load_tuning("resnet50", 4))
    fv, fi = fresh.classify(torch.from_numpy(x).cuda(), 5)
    np.testing.assert_array_equal(i1, fi.cpu().numpy())
    np.testing.assert_allclose(v1, fv.cpu().numpy(), rtol=1e-3, atol=1e-4)
    assert not np.array_equal(i0, i1)


class _Part:
    def __init__(self, data: bytes):
        self.data, self.content_type = data, "application/octet-stream"


def test_resnet50_auto_batch_plan():
    """MAX_BATCH=0: the cap is planned from measured activation bytes / time, free HBM and the SLO."""
    from mlmicroservicetemplate_amd.config import Settings
    from mlmicroservicetemplate_amd.plugins.base import PluginContext
    from mlmicroservicetemplate_amd.plugins.builtin import ResNet50Plugin

    s = Settings.load(env_file=None, environ={}, overrides={"REGISTER": False, "GPUS": 1, "MODEL": "resnet50",
                                                            "MAX_BATCH": 0, "LATENCY_SLO_MS": 3.0, "INFLIGHT": 2})
    plugin = ResNet50Plugin()
    plugin.init(PluginContext(settings=s, devices=["cuda:0"]))
    plan = plugin.capacity_plan
    assert plan.limit == "slo" and 1 <= plan.max_batch <= 1024  # 288 GB never binds for ResNet-50
    assert plan.per_sample_bytes > 1e5 and plan.free_bytes > 1e11
    assert s.MAX_BATCH == plan.max_batch and s.GRAPH_BUCKETS[-1] == plan.max_batch
    assert plugin.engines[0].max_batch == plan.max_batch
    x = np.random.default_rng(0).integers(0, 256, (plan.max_batch, 224, 224, 3), dtype=np.uint8)
    v, i = plugin.engines[0].run(np.stack([plugin.preprocess(_Part(img.tobytes())) for img in x]))
    assert v.shape == (plan.max_batch, 5) and np.all(np.isfinite(v))
