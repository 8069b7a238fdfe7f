"""Registration heartbeat client (reference server_connection.py:10-34) against an in-process
fake orchestrator."""
import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


from mlmicroservicetemplate_amd.api.state import ServiceState
from mlmicroservicetemplate_amd.discovery import register_model_to_server, registration_payload


class FakeOrchestrator:
    def __init__(self, fail_first=0, status=200, delay=0.0):
        self.requests = []
        self.fail_first = fail_first
        self.status = status
        self.delay = delay
        outer = self

        class H(BaseHTTPRequestHandler):
            def do_POST(self):
                n = int(self.headers.get("content-length", 0))
                body = json.loads(self.rfile.read(n))
                outer.requests.append((self.path, dict(self.headers), body, time.time()))
                if outer.delay:
                    time.sleep(outer.delay)
                code = 500 if len(outer.requests) <= outer.fail_first else outer.status
                self.send_response(code)
                self.end_headers()

            def log_message(self, *a):
                pass

        self.server = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.port = self.server.server_address[1]
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True)
        self.thread.start()

    def close(self):
        self.server.shutdown()
        self.server.server_close()


def run_hb(state, port, **kw):
    args = dict(api_key="k3y", server_host="127.0.0.1", advertise_host="host.docker.internal", wait_time=0.05,
                timeout=1.0)
    args.update(kw)
    t = threading.Thread(target=register_model_to_server, args=(state, port, 5005, "example_model"), kwargs=args)
    t.start()
    return t


def test_payload_and_heartbeat_cadence():
    orch = FakeOrchestrator()
    state = ServiceState(pool_workers=1)
    t = run_hb(state, orch.port)
    time.sleep(0.4)
    state.shutdown.set()
    t.join(2)
    orch.close()
    assert not t.is_alive()
    assert len(orch.requests) >= 3  # keeps re-registering (heartbeat), not one-shot
    path, headers, body, _ = orch.requests[0]
    assert path == "/model/register"
    assert headers.get("api_key") == "k3y"
    assert body == {"name": "example_model", "socket": "http://host.docker.internal:5005"}
    assert state.connected is True


def test_retry_on_http_error_then_success():
    orch = FakeOrchestrator(fail_first=2)
    state = ServiceState(pool_workers=1)
    seen = []
    t = run_hb(state, orch.port, on_attempt=seen.append)
    time.sleep(0.35)
    state.shutdown.set()
    t.join(2)
    orch.close()
    assert seen[:3] == [False, False, True]
    assert state.connected


def test_connection_refused_keeps_retrying_and_stops_promptly():
    state = ServiceState(pool_workers=1)
    seen = []
    t = run_hb(state, 1, on_attempt=seen.append, wait_time=5.0)  # port 1: refused
    time.sleep(0.2)
    t0 = time.time()
    state.shutdown.set()
    t.join(2)
    assert not t.is_alive() and time.time() - t0 < 1.0  # Event wait wakes immediately
    assert seen and not any(seen) and state.connected is False


def test_hung_orchestrator_does_not_block_shutdown():
    orch = FakeOrchestrator(delay=3.0)
    state = ServiceState(pool_workers=1)
    t = run_hb(state, orch.port, timeout=0.2)
    time.sleep(0.3)
    state.shutdown.set()
    t.join(1.5)
    assert not t.is_alive()
    orch.close()


def test_invalid_url_does_not_kill_thread():
    state = ServiceState(pool_workers=1)
    seen = []
    t = run_hb(state, None, server_host="bad host name with spaces", on_attempt=seen.append)
    time.sleep(0.2)
    state.shutdown.set()
    t.join(2)
    assert len(seen) >= 2  # still looping after the InvalidURL


def test_legacy_payload():
    assert registration_payload("m", "h", 5005, legacy=True) == {"modelName": "m", "modelPort": 5005}


def test_legacy_payload_via_settings():
    """REGISTER_LEGACY=1 makes the heartbeat send the old-rev body without the api_key header."""
    from mlmicroservicetemplate_amd.config import Settings
    from mlmicroservicetemplate_amd.discovery import start_heartbeat

    orch = FakeOrchestrator()
    s = Settings.load(env_file=None, environ={"SERVER_PORT": str(orch.port), "SERVER_HOST": "127.0.0.1",
                                               "REGISTER_LEGACY": "1", "HEARTBEAT_S": "0.05", "API_KEY": "k3y"})
    state = ServiceState(pool_workers=1)
    start_heartbeat(state, s)
    deadline = time.time() + 5
    while not orch.requests and time.time() < deadline:
        time.sleep(0.02)
    state.begin_shutdown(wait=True)
    orch.close()
    path, headers, body, _ = orch.requests[0]
    assert path == "/model/register"
    assert body == {"modelName": s.NAME, "modelPort": s.PORT}
    assert "api_key" not in {k.lower() for k in headers}
