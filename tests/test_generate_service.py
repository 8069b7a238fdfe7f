"""/generate end to end on CPU: tiny Llama, single process and TP=2 (two ranks over gloo,
rank 0 serving HTTP and broadcasting commands), same greedy tokens as the in-process model."""
import os
import signal
import socket
import subprocess
import sys
import time
import warnings

import pytest
import requests
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
warnings.filterwarnings("ignore", category=DeprecationWarning)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _yaml(tmp_path):
    y = tmp_path / "llama.yaml"
    y.write_text("config: tiny\nmax_seq: 128\noverrides:\n  layers: 2\n")
    return str(y)


def _expected(prompt_ids, n):
    from mlmicroservicetemplate_amd.models.llama import GenParams, LlamaTP, init_llama_shard, tiny_config

    cfg = tiny_config(layers=2)
    m = LlamaTP(init_llama_shard(cfg, 1, 0, seed=0), cfg, max_batch=8, max_seq=128)
    return m.generate(torch.tensor([prompt_ids]), torch.tensor([len(prompt_ids)]), GenParams(n))[0].tolist()


def test_generate_in_process(tmp_path):
    from fastapi.testclient import TestClient

    from mlmicroservicetemplate_amd.api.app import create_app
    from mlmicroservicetemplate_amd.config import Settings

    s = Settings.load(env_file=None, environ={}, overrides={"REGISTER": False, "MODEL": "llama",
                                                          "MODEL_CONFIG": _yaml(tmp_path), "MAX_BATCH": 8,
                                                          "GPUS": 0})
    with TestClient(create_app(s), raise_server_exceptions=False) as c:
        t0 = time.time()
        while c.get("/status").status_code != 200 and time.time() - t0 < 60:
            time.sleep(0.05)
        ids = [1, 55, 99, 1000]
        r = c.post("/generate", json={"input_ids": ids, "max_new_tokens": 5})
        assert r.status_code == 200, r.text
        res = r.json()["result"]
        assert res["token_ids"] == _expected(ids, 5)[: res["num_tokens"]]
        assert res["prompt_tokens"] == 4
        r = c.post("/generate", json={"prompt": "hello MI355X world", "max_new_tokens": 3, "top_k": 5, "seed": 1})
        assert r.status_code == 200 and r.json()["result"]["num_tokens"] <= 3
        assert c.post("/generate", json={"input_ids": [], "max_new_tokens": 3}).status_code == 400
        assert c.post("/predict").status_code == 422


@pytest.mark.timeout(180)
def test_generate_tp2_service(tmp_path):
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               MODEL_CONFIG=_yaml(tmp_path), LOG_LEVEL="warning")
    proc = subprocess.Popen([sys.executable, "-m", "mlmicroservicetemplate_amd", "serve", "--model", "llama", "--tp", "2",
                             "--port", str(port), "--host", "127.0.0.1", "--no-register", "--env-file", "/nonexistent"],
                            cwd=ROOT, env=env, start_new_session=True)
    try:
        url = f"http://127.0.0.1:{port}"
        deadline = time.time() + 120
        while time.time() < deadline:
            try:
                if requests.get(url + "/status", timeout=1).status_code == 200:
                    break
            except requests.RequestException:
                pass
            time.sleep(0.3)
        ids = [1, 55, 99, 1000]
        exp = _expected(ids, 6)
        for _ in range(2):
            r = requests.post(url + "/generate", json={"input_ids": ids, "max_new_tokens": 6}, timeout=60)
            assert r.status_code == 200, r.text
            res = r.json()["result"]
            assert res["token_ids"] == exp[: res["num_tokens"]]
        info = requests.get(url + "/info", timeout=5).json()
        assert info["model"]["tp"] == 2
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
