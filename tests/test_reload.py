"""Hot weight reload (POST /admin/reload, parallel/reload.py) on CPU with the toy classifier:
both front ends, auth, errors, safetensors source, and the 2-rank (gloo) broadcast path."""
import os
import signal
import socket
import subprocess
import sys
import time
import warnings

import numpy as np
import pytest
import requests

warnings.filterwarnings("ignore", category=DeprecationWarning)

from fastapi.testclient import TestClient  # noqa: E402

from mlmicroservicetemplate_amd.api.app import create_app  # noqa: E402
from mlmicroservicetemplate_amd.api.multipart import encode_multipart  # noqa: E402
from mlmicroservicetemplate_amd.config import Settings  # noqa: E402
from mlmicroservicetemplate_amd.frontend.native import NativeService  # noqa: E402
from mlmicroservicetemplate_amd.plugins.base import PluginContext  # noqa: E402
from mlmicroservicetemplate_amd.plugins.builtin import ToyClassifierPlugin  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def settings(**kw):
    base = {"MODEL": "toy_classifier", "REGISTER": False, "MAX_WAIT_US": 2000, "IO_THREADS": 2}
    base.update(kw)
    return Settings.load(env_file=None, environ={}, overrides=base)


def img(seed=0):
    return np.random.default_rng(seed).integers(0, 256, (8, 8, 3), dtype=np.uint8)


def upload(a):
    body, ct = encode_multipart({"image_file": ("x.rgb", a.tobytes(), "application/octet-stream")})
    return body, {"content-type": ct}


def expected_classes(seed, a):
    p = ToyClassifierPlugin()
    p.w = p.load_params(None, seed)["w"].numpy()
    _, idx = p.scores(a[None])
    return [f"class_{i}" for i in idx[0]]


def _ready(get, timeout=10):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if get("/status").status_code == 200:
            return True
        time.sleep(0.01)
    return False


def test_reload_python_frontend_seed_auth_and_errors(tmp_path):
    a = img(1)
    with TestClient(create_app(settings(API_KEY="sekret", WEIGHTS_DIR=str(tmp_path)), ToyClassifierPlugin())) as c:
        assert _ready(c.get)
        body, h = upload(a)
        assert c.post("/predict", content=body, headers=h).json()["result"]["classes"] == expected_classes(0, a)
        assert c.post("/admin/reload", json={"seed": 3}).status_code == 401
        assert c.post("/admin/reload", json={"seed": 3}, headers={"api_key": "nope"}).status_code == 401
        r = c.post("/admin/reload", json={"seed": 3}, headers={"api_key": "sekret"})
        assert r.status_code == 200 and r.json()["result"]["generation"] == 1
        assert c.post("/predict", content=body, headers=h).json()["result"]["classes"] == expected_classes(3, a)
        bad = c.post("/admin/reload", json={"weights": str(tmp_path / "missing.safetensors")}, headers={"api_key": "sekret"})
        assert bad.status_code == 400 and "under WEIGHTS_DIR" in bad.json()["detail"]
        # a file that exists outside WEIGHTS_DIR gets the same answer (no path-existence oracle)
        outside = c.post("/admin/reload", json={"weights": os.path.abspath(__file__)}, headers={"api_key": "sekret"})
        assert outside.status_code == 400 and outside.json()["detail"] == bad.json()["detail"]
        dotdot = c.post("/admin/reload", json={"weights": "../" + os.path.basename(str(tmp_path))}, headers={"api_key": "sekret"})
        assert dotdot.status_code == 400 and dotdot.json()["detail"] == bad.json()["detail"]
        assert c.post("/admin/reload", json={}, headers={"api_key": "sekret"}).status_code == 400
        # safetensors source, validated against the plugin's spec
        from mlmicroservicetemplate_amd.utils.checkpoint import save_state

        path = str(tmp_path / "toy.safetensors")
        save_state(path, ToyClassifierPlugin().load_params(None, 11))
        r = c.post("/admin/reload", json={"weights": "toy.safetensors"}, headers={"api_key": "sekret"})
        assert r.status_code == 200 and r.json()["result"]["generation"] == 2
        r = c.post("/admin/reload", json={"weights": path}, headers={"api_key": "sekret"})  # absolute, inside
        assert r.status_code == 200 and r.json()["result"]["generation"] == 3
        assert c.post("/predict", content=body, headers=h).json()["result"]["classes"] == expected_classes(11, a)


def test_reload_disabled_without_api_key(tmp_path):
    """No API_KEY configured: /admin/reload is refused on both front ends (403) and the weights
    are untouched."""
    a = img(1)
    with TestClient(create_app(settings(WEIGHTS_DIR=str(tmp_path)), ToyClassifierPlugin())) as c:
        assert _ready(c.get)
        body, h = upload(a)
        r = c.post("/admin/reload", json={"seed": 3})
        assert r.status_code == 403 and "API_KEY" in r.json()["detail"]
        assert c.post("/admin/reload", json={"seed": 3}, headers={"api_key": ""}).status_code == 403
        assert c.post("/predict", content=body, headers=h).json()["result"]["classes"] == expected_classes(0, a)
    s = settings()
    svc = NativeService(s, ToyClassifierPlugin(), PluginContext(settings=s), host="127.0.0.1", port=0).start()
    try:
        url = f"http://127.0.0.1:{svc.port}"
        assert _ready(lambda p: requests.get(url + p))
        assert requests.post(url + "/admin/reload", json={"seed": 5}).status_code == 403
        assert requests.post(url + "/predict", data=body, headers=h).json()["result"]["classes"] == expected_classes(0, a)
    finally:
        svc.stop()


def test_reload_native_frontend():
    a = img(2)
    s = settings(API_KEY="k")
    svc = NativeService(s, ToyClassifierPlugin(), PluginContext(settings=s), host="127.0.0.1", port=0).start()
    try:
        url = f"http://127.0.0.1:{svc.port}"
        assert _ready(lambda p: requests.get(url + p))
        body, h = upload(a)
        assert requests.post(url + "/predict", data=body, headers=h).json()["result"]["classes"] == expected_classes(0, a)
        r = requests.post(url + "/admin/reload", json={"seed": 5}, headers={"api_key": "k"})
        assert r.status_code == 200 and r.json()["result"]["ranks"] == 1
        assert requests.post(url + "/predict", data=body, headers=h).json()["result"]["classes"] == expected_classes(5, a)
        assert requests.get(url + "/admin/reload").status_code == 405
    finally:
        svc.stop()


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


@pytest.mark.timeout(150)
@pytest.mark.parametrize("frontend", ["python", "native"])
def test_reload_two_ranks_broadcasts_to_every_rank(frontend):
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", API_KEY="k")
    proc = subprocess.Popen([sys.executable, "-m", "mlmicroservicetemplate_amd", "serve", "--model", "toy_classifier",
                             "--frontend", frontend, "--gpus", "2", "--port", str(port), "--host", "127.0.0.1",
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
        key = {"api_key": "k"}
        # /status answered by one rank does not mean the other (sharing the port) is ready yet
        for _ in range(150):
            r = requests.post(url + "/admin/reload", json={"seed": 7}, headers=key, timeout=60)
            if r.status_code != 503:
                break
            time.sleep(0.2)
        assert r.status_code == 200, r.text
        assert r.json()["result"]["ranks"] == 2
        # two reloads racing (fresh connections may land on different ranks): the ranks must stay
        # in step -- each request is applied by every rank or refused with 409, never skipped
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(4) as ex:
            codes = [f.result().status_code for f in
                     [ex.submit(requests.post, url + "/admin/reload", json={"seed": 8}, headers=key, timeout=60)
                      for _ in range(4)]]
        assert set(codes) <= {200, 409} and 200 in codes, codes
        # back to back: the group is not wedged and both ranks apply the final generation
        r = requests.post(url + "/admin/reload", json={"seed": 9}, headers=key, timeout=60)
        assert r.status_code == 200, r.text
        assert r.json()["result"]["ranks"] == 2
        a = img(4)
        want = expected_classes(9, a)
        body, h = upload(a)
        ranks = set()
        # fresh connections land on both ranks; every rank serves the new weights.  SO_REUSEPORT spreads
        # new connections by hash, and under a loaded CPU (parallel test workers) a rank can miss a
        # burst of them, so the loop paces itself instead of relying on 60 back-to-back tries
        for i in range(400):
            ranks.add(requests.get(url + "/info", timeout=5).json()["rank"])
            assert requests.post(url + "/predict", data=body, headers=h, timeout=5).json()["result"]["classes"] == want
            if len(ranks) == 2:
                break
            if i >= 40:
                time.sleep(0.05)
        assert ranks == {0, 1}
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)


def test_control_dir_refuses_symlinks_foreign_modes(tmp_path):
    """the reload control directory is trusted by every rank, so it must be a 0700
    directory of ours -- never a symlink or a group/world-writable directory someone pre-created."""
    from mlmicroservicetemplate_amd.parallel.reload import secure_control_dir

    d = secure_control_dir(str(tmp_path / "ctl"))
    assert (os.stat(d).st_mode & 0o777) == 0o700
    assert secure_control_dir(d) == d  # a second rank of the same launch reuses it
    target = tmp_path / "elsewhere"
    target.mkdir(mode=0o700)
    os.symlink(target, tmp_path / "link")
    with pytest.raises(PermissionError):
        secure_control_dir(str(tmp_path / "link"))
    loose = tmp_path / "loose"
    loose.mkdir()
    os.chmod(loose, 0o777)
    with pytest.raises(PermissionError):
        secure_control_dir(str(loose))


class _FakePlugin:
    name = "fake"

    def __init__(self):
        self.applied = []

    def reload_spec(self):
        return {}

    def load_params(self, weights, seed):
        return {}

    def apply_params(self, params):
        self.applied.append(params)


def test_stale_generation_is_replaced_and_watcher_acks_failures(tmp_path, monkeypatch):
    """A generation some rank never acknowledged blocks new ones (409) only until the request
    timeout has passed; a watcher whose apply raises writes an error ack instead of dying."""
    import json
    import time
    from types import SimpleNamespace

    from mlmicroservicetemplate_amd.parallel import reload as rl

    monkeypatch.setenv("MLS_RELOAD_BASE", str(tmp_path))
    monkeypatch.setenv("MLS_LAUNCH_ID", "testlaunch")
    ctx = SimpleNamespace(rank=1, world_size=2)
    settings = SimpleNamespace(PORT=1, WEIGHTS_DIR="")
    co = rl.ReloadCoordinator(_FakePlugin(), ctx, settings, poll_s=0.01)
    try:
        assert co.ctl_dir.startswith(str(tmp_path)) and co.ctl_dir.endswith("-testlaunch")
        # the watcher (rank 1) will fail to apply: there is no process group here
        req = os.path.join(co.ctl_dir, "request.json")
        rl._atomic_write(req, {"generation": 1, "seed": 3, "t": time.time(), "timeout": 0.3})
        ack = os.path.join(co.ctl_dir, "ack-1-1.json")
        for _ in range(300):
            if os.path.exists(ack):
                break
            time.sleep(0.01)
        a = json.load(open(ack))
        assert a["generation"] == 1 and a["error"]
        assert co._thread.is_alive()  # the watcher survived its failed generation
        # rank 0 never acked generation 1: a new request is refused until it is stale
        co._stop.set()
        co._thread.join(2)
        with pytest.raises(rl.ReloadBusy):
            co.request(seed=4, timeout=0.3)
        time.sleep(0.35)
        with pytest.raises(TimeoutError):  # accepted as generation 2 (no rank applies it here)
            co.request(seed=4, timeout=0.2)
        assert json.load(open(req))["generation"] == 2
    finally:
        co.close()


def test_respawned_replica_refuses_reload(tmp_path, monkeypatch):
    """A DP replica restarted by serve.py runs standalone (WORLD_SIZE=1, no control dir): it must
    answer 409 like the surviving replicas instead of loading weights only it would serve
    (serve._respawn_env sets MLS_RESPAWNED_REPLICA)."""
    from mlmicroservicetemplate_amd import serve

    env = serve._respawn_env({"WORLD_SIZE": "4", "MASTER_PORT": "1"}, 2, None, settings())
    assert env["MLS_RESPAWNED_REPLICA"] == "1" and env["WORLD_SIZE"] == "1"
    monkeypatch.setenv("MLS_RESPAWNED_REPLICA", "1")
    a = img(1)
    with TestClient(create_app(settings(API_KEY="sekret", WEIGHTS_DIR=str(tmp_path)), ToyClassifierPlugin())) as c:
        assert _ready(c.get)
        r = c.post("/admin/reload", json={"seed": 3}, headers={"api_key": "sekret"})
        assert r.status_code == 409 and "restarted" in r.json()["detail"]
        body, h = upload(a)  # still serving the weights it started with
        assert c.post("/predict", content=body, headers=h).json()["result"]["classes"] == expected_classes(0, a)
