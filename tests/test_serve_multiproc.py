"""Launcher: 2 ranks (gloo on CPU) sharing one port via SO_REUSEPORT, identity model."""
import os
import signal
import socket
import subprocess
import sys
import time

import pytest
import requests

from mlmicroservicetemplate_amd.api.multipart import encode_multipart

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(120)
def test_two_rank_identity_service():
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    proc = subprocess.Popen([sys.executable, "-m", "mlmicroservicetemplate_amd", "serve", "--model", "identity",
                             "--gpus", "2", "--port", str(port), "--host", "127.0.0.1", "--no-register",
                             "--env-file", "/nonexistent"], cwd=ROOT, env=env, start_new_session=True)
    try:
        url = f"http://127.0.0.1:{port}"
        deadline = time.time() + 90
        ready = False
        while time.time() < deadline:
            try:
                if requests.get(url + "/status", timeout=1).status_code == 200:
                    ready = True
                    break
            except requests.RequestException:
                pass
            time.sleep(0.2)
        assert ready, "service never became ready"
        ranks = set()
        for i in range(40):
            info = requests.get(url + "/info", timeout=5).json()
            ranks.add(info["rank"])
            assert info["world_size"] == 2
            body, ct = encode_multipart({"image_file": ("x", os.urandom(64), "application/octet-stream")})
            r = requests.post(url + "/predict", data=body, headers={"content-type": ct}, timeout=5)
            assert r.status_code == 200 and r.json()["result"]["result"]["bytes"] == 64
            if len(ranks) == 2:
                break
        assert ranks == {0, 1}, f"SO_REUSEPORT did not spread connections: {ranks}"
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)


@pytest.mark.timeout(120)
def test_workers_per_gpu_share_the_port():
    """WORKERS_PER_GPU: independent serving processes on one port (front-end CPU scaling)."""
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    proc = subprocess.Popen([sys.executable, "-m", "mlmicroservicetemplate_amd", "serve", "--model", "identity",
                             "--workers-per-gpu", "3", "--port", str(port), "--host", "127.0.0.1", "--no-register",
                             "--env-file", "/nonexistent"], cwd=ROOT, env=env, start_new_session=True)
    try:
        url = f"http://127.0.0.1:{port}"
        deadline = time.time() + 90
        pids, workers = set(), set()
        while time.time() < deadline and len(workers) < 3:
            try:
                if requests.get(url + "/status", timeout=1).status_code != 200:
                    time.sleep(0.1)
                    continue
                h = requests.get(url + "/health", timeout=2).json()
                pids.add(h["pid"])
                workers.add(h["worker"])
                body, ct = encode_multipart({"image_file": ("x", b"abc", "application/octet-stream")})
                r = requests.post(url + "/predict", data=body, headers={"content-type": ct}, timeout=5)
                assert r.status_code == 200
            except requests.RequestException:
                time.sleep(0.1)
        assert workers == {0, 1, 2} and len(pids) == 3, (workers, pids)
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)


@pytest.mark.timeout(240)
def test_dp_replica_fault_isolation_and_restart():
    """in DP serving a dead replica must not take the others down.  3 identity
    ranks; one is SIGKILLed after start-up; /status and /predict keep answering 200 from the
    survivors throughout, and the supervisor's fresh replacement process serves again."""
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    proc = subprocess.Popen([sys.executable, "-m", "mlmicroservicetemplate_amd", "serve", "--model", "identity",
                             "--gpus", "3", "--port", str(port), "--host", "127.0.0.1", "--no-register",
                             "--env-file", "/nonexistent"], cwd=ROOT, env=env, start_new_session=True)
    url = f"http://127.0.0.1:{port}"

    def predict():
        body, ct = encode_multipart({"image_file": ("x", b"abcd", "application/octet-stream")})
        return requests.post(url + "/predict", data=body, headers={"content-type": ct, "connection": "close"},
                             timeout=5)

    try:
        deadline = time.time() + 120
        pids = set()
        while time.time() < deadline and len(pids) < 3:
            try:
                h = requests.get(url + "/health", headers={"connection": "close"}, timeout=2).json()
                if requests.get(url + "/status", headers={"connection": "close"}, timeout=2).status_code == 200:
                    pids.add(h["pid"])
            except requests.RequestException:
                pass
            time.sleep(0.05)
        assert len(pids) == 3, f"not every rank became ready: {pids}"
        victim = sorted(pids)[1]
        os.kill(victim, signal.SIGKILL)
        # the survivors answer throughout: every probe is 200 (no 503 window, no refused connection)
        new_pids, t_end = set(), time.time() + 150
        while time.time() < t_end:
            st = requests.get(url + "/status", headers={"connection": "close"}, timeout=5)
            assert st.status_code == 200, st.text
            r = predict()
            assert r.status_code == 200 and r.json()["result"]["result"]["bytes"] == 4
            h = requests.get(url + "/health", headers={"connection": "close"}, timeout=5).json()
            assert h["pid"] != victim
            if h["pid"] not in pids:
                new_pids.add(h["pid"])
                break
            time.sleep(0.02)
        assert new_pids, "the replacement replica never served"
        assert proc.poll() is None, "the supervisor exited"
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
