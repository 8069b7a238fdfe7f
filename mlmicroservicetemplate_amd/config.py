"""Typed service configuration (T0).

Reference behaviour:
  * ``.env`` holds ``NAME`` / ``PORT`` / ``SERVER_PORT`` (reference ``.env:1-3``) and is read at
    startup with ``load_dotenv()`` + ``os.getenv`` (reference ``src/server/main.py:72,82``).
  * the API key lives in a repo-root module called ``secrets`` (reference ``secrets.py:2``) --
    which shadows the stdlib module; here it comes from ``API_KEY`` (env / .env) or
    ``API_KEY_FILE`` instead, never from a module named ``secrets``.
  * hard-coded knobs: pool size 10 (``dependency.py:19``), heartbeat 10 s (``dependency.py:20``),
    CORS origins (``main.py:22-28``).

Here every knob is one field of :class:`Settings`, resolved with precedence
``defaults < .env file < process environment < explicit overrides``.  python-dotenv and
pydantic-settings are not installed, so the ``.env`` parser is in-house.
"""
from __future__ import annotations

import dataclasses
import os
import re
from dataclasses import dataclass, field
from typing import Any, Dict, List, Mapping, Optional, Tuple

DEFAULT_CORS_ORIGINS: Tuple[str, ...] = (
    "http://localhost",
    "http://localhost:3000",
    "http://localhost:5057",
    "http://localhost:5000",
    "http://localhost:6379",
)

_LINE = re.compile(
    r"""^\s*(?:export\s+)?(?P<key>[A-Za-z_][A-Za-z0-9_.]*)\s*(?:=\s*(?P<val>.*?))?\s*$"""
)


def _unquote(raw: str) -> str:
    raw = raw.strip()
    if len(raw) >= 2 and raw[0] == raw[-1] and raw[0] in "'\"":
        body = raw[1:-1]
        if raw[0] == '"':
            body = (
                body.replace("\\n", "\n").replace("\\t", "\t").replace('\\"', '"').replace("\\\\", "\\")
            )
        return body
    # strip an inline comment: `KEY=value # comment` (a '#' glued to text is kept)
    m = re.search(r"\s+#", raw)
    if m:
        raw = raw[: m.start()]
    return raw.strip()


def _expand(value: str, scope: Mapping[str, str]) -> str:
    """``${VAR}`` / ``${VAR:-default}`` interpolation, as docker-compose does for the same file."""

    def sub(m: "re.Match[str]") -> str:
        name, default = m.group(1), m.group(3)
        got = scope.get(name)
        if got is None or (got == "" and m.group(2) == ":-"):
            return default or ""
        return got

    return re.sub(r"\$\{([A-Za-z_][A-Za-z0-9_]*)(?:(:?-)([^}]*))?\}", sub, value)


def parse_dotenv(text: str, environ: Optional[Mapping[str, str]] = None) -> Dict[str, str]:
    """Parse dotenv text into a dict.  Supports comments, ``export``, single/double quotes,
    multi-line double-quoted values, inline comments and ``${VAR}`` interpolation."""
    out: Dict[str, str] = {}
    lines = text.splitlines()
    i = 0
    while i < len(lines):
        line = lines[i]
        i += 1
        if not line.strip() or line.lstrip().startswith("#"):
            continue
        m = _LINE.match(line)
        if not m:
            continue
        key, val = m.group("key"), m.group("val")
        if val is None:
            continue
        # multi-line double-quoted value
        if val.startswith('"') and (val.count('"') - val.count('\\"')) % 2 == 1:
            parts = [val]
            while i < len(lines):
                parts.append(lines[i])
                i += 1
                if lines[i - 1].rstrip().endswith('"'):
                    break
            val = "\n".join(parts)
        quoted_single = val.strip().startswith("'")
        val = _unquote(val)
        if not quoted_single:
            scope = dict(environ or {})
            scope.update(out)
            val = _expand(val, scope)
        out[key] = val
    return out


def load_dotenv(path: str = ".env", override: bool = False, environ=None) -> Dict[str, str]:
    """Drop-in for ``dotenv.load_dotenv``: read ``path`` and export keys into ``environ``
    (default ``os.environ``) without overriding existing variables unless ``override``."""
    environ = os.environ if environ is None else environ
    if not os.path.isfile(path):
        return {}
    with open(path, "r", encoding="utf-8") as f:
        values = parse_dotenv(f.read(), environ)
    for k, v in values.items():
        if override or k not in environ:
            environ[k] = v
    return values


def _to_bool(v: Any) -> bool:
    if isinstance(v, bool):
        return v
    return str(v).strip().lower() in ("1", "true", "yes", "on", "y")


def _to_list(v: Any, item=str) -> list:
    if isinstance(v, (list, tuple)):
        return [item(x) for x in v]
    s = str(v).strip()
    if not s:
        return []
    return [item(x.strip()) for x in s.split(",") if x.strip()]


@dataclass
class Settings:
    """All service knobs.  Field name == environment variable name."""

    # --- reference keys (.env:1-3, secrets.py:2) ---
    NAME: str = "example_model"
    PORT: int = 5005
    SERVER_PORT: Optional[int] = 5000
    API_KEY: str = ""
    # --- discovery (server_connection.py:20-22) ---
    SERVER_HOST: str = "host.docker.internal"
    ADVERTISE_HOST: str = "host.docker.internal"
    REGISTER: bool = True
    HEARTBEAT_S: float = 10.0  # dependency.WAIT_TIME
    REGISTER_TIMEOUT_S: float = 5.0  # the reference had none (a hung POST blocked shutdown)
    REGISTER_LEGACY: bool = False  # old-rev {"modelName","modelPort"} body, no api_key header
    POOL_WORKERS: int = 10  # dependency.pool size
    # --- model / plugin ---
    MODEL: str = "stub"  # stub | identity | resnet50 | bert | llama | <python.module.path>
    MODEL_CONFIG: str = ""  # optional YAML with per-model overrides
    BACKEND: str = "fused"  # fused (our HIP kernels) | eager (stock torch) | reference (fp32)
    DTYPE: str = "bf16"
    SEED: int = 0
    WEIGHTS: str = ""  # optional .safetensors path
    WEIGHTS_DIR: str = ""  # POST /admin/reload may only load safetensors under this directory ("" = seed reloads only)
    IMAGE_DIR: str = "src/images"  # legacy /predict?filename= flow (old-rev main.pyc@L119-152)
    TOPK: int = 5
    # image models: uploads become GPU image containers -- baseline JPEGs Huffman-decoded on the host
    # (C++), IDCT / colour / resize on the GPU inside the serving graph (ops.image_decode)
    GPU_IMAGE_DECODE: bool = True
    # --- GPU execution ---
    GPUS: int = 1
    WORKERS_PER_GPU: int = 1  # HTTP worker processes per GPU (DP models): front-end CPU scales, each owns an engine
    TP: int = 1
    MAX_BATCH: int = 32  # 0 = auto: planned from free HBM / per-sample activations and LATENCY_SLO_MS
    MAX_BATCH_CAP: int = 1024  # ceiling of an auto-planned batch
    LATENCY_SLO_MS: float = 50.0  # auto planning: GPU time budget of one batch
    MAX_WAIT_US: int = 2000
    MAX_QUEUE: int = 4096
    GRAPH_BUCKETS: List[int] = field(default_factory=lambda: [1, 2, 4, 8, 16, 32])
    USE_GRAPHS: bool = True
    INFLIGHT: int = 5  # batches in flight per GPU worker: H2D/compute/D2H overlap + co-running graphs (r1 sweep)
    CONCURRENT_SLOTS: bool = True  # in-flight batches co-run on per-slot streams (+26 % ResNet-50 req/s)
    CU_PARTITION: int = 2  # ResNet-50 engine: slot streams CU-masked into this many halves (0 = off; engine/worker.py)
    REQUEST_TIMEOUT_S: float = 30.0
    WATCHDOG_INTERVAL_S: float = 1.0  # replica liveness check period (0 disables the watchdog)
    WATCHDOG_STALL_S: float = 30.0  # a batch running longer than this drains its replica
    WATCHDOG_MAX_FAILURES: int = 3  # consecutive failed batches that drain a replica
    WATCHDOG_COOLDOWN_S: float = 30.0  # failure-drained replica re-admitted on probation after this
    HBM_FRACTION: float = 0.9  # of free HBM the batch-size cap may plan for
    # --- generate (Llama) ---
    MAX_NEW_TOKENS: int = 64
    CONTINUOUS_BATCHING: bool = True  # /generate: sequences join / leave the decode batch every step
    MAX_SEQ_LEN: int = 8192
    # --- HTTP ---
    FRONTEND: str = "python"  # python (FastAPI/uvicorn) | native (C++ epoll server + C++ batcher)
    IO_THREADS: int = 4  # native front end: epoll I/O threads per serving process
    DECODE_WORKERS: int = 4  # native front end: Python threads decoding non-raw uploads (JPEG/PNG)
    CORS_ORIGINS: List[str] = field(default_factory=lambda: list(DEFAULT_CORS_ORIGINS))
    MAX_UPLOAD_BYTES: int = 64 * 1024 * 1024
    LOG_LEVEL: str = "info"

    _env_file: str = ".env"

    @classmethod
    def field_names(cls) -> List[str]:
        return [f.name for f in dataclasses.fields(cls) if not f.name.startswith("_")]

    @classmethod
    def load(
        cls,
        env_file: Optional[str] = ".env",
        environ: Optional[Mapping[str, str]] = None,
        overrides: Optional[Mapping[str, Any]] = None,
    ) -> "Settings":
        environ = dict(os.environ if environ is None else environ)
        merged: Dict[str, Any] = {}
        if env_file and os.path.isfile(env_file):
            with open(env_file, "r", encoding="utf-8") as f:
                merged.update(parse_dotenv(f.read(), environ))
        names = set(cls.field_names())
        for k, v in environ.items():
            if k in names:
                merged[k] = v
        for k, v in (overrides or {}).items():
            if v is not None:
                merged[k] = v
        if not merged.get("API_KEY") and merged.get("API_KEY_FILE", environ.get("API_KEY_FILE")):
            with open(merged.get("API_KEY_FILE") or environ["API_KEY_FILE"], encoding="utf-8") as f:
                merged["API_KEY"] = f.read().strip()
        s = cls()
        s._env_file = env_file or ""
        for f in dataclasses.fields(cls):
            if f.name.startswith("_") or f.name not in merged:
                continue
            setattr(s, f.name, cls._coerce(f, merged[f.name]))
        s.validate()
        return s

    @staticmethod
    def _coerce(f: dataclasses.Field, v: Any) -> Any:
        t = f.type if isinstance(f.type, str) else getattr(f.type, "__name__", str(f.type))
        if v is None:
            return None
        if t in ("int",):
            return int(v)
        if t in ("float",):
            return float(v)
        if t in ("bool",):
            return _to_bool(v)
        if t.startswith("Optional[int]"):
            return None if str(v).strip() in ("", "None", "none", "null") else int(v)
        if t.startswith("List[int]"):
            return _to_list(v, int)
        if t.startswith("List[str]"):
            return _to_list(v, str)
        return str(v)

    def validate(self) -> None:
        if not (0 < self.PORT < 65536):
            raise ValueError(f"PORT out of range: {self.PORT}")
        if self.MAX_BATCH < 0:
            raise ValueError("MAX_BATCH must be >= 1, or 0 for an HBM / latency-planned batch")
        if self.GPUS < 0 or self.TP < 1:
            raise ValueError("GPUS must be >= 0 and TP >= 1")
        if self.DTYPE not in ("bf16", "fp32", "fp16"):
            raise ValueError(f"unsupported DTYPE {self.DTYPE}")
        if self.FRONTEND not in ("python", "native"):
            raise ValueError(f"FRONTEND must be python or native, not {self.FRONTEND!r}")
        self.GRAPH_BUCKETS = sorted(set(int(b) for b in self.GRAPH_BUCKETS if int(b) > 0))
        if self.MAX_BATCH and (not self.GRAPH_BUCKETS or self.GRAPH_BUCKETS[-1] < self.MAX_BATCH):
            self.GRAPH_BUCKETS = sorted(set(self.GRAPH_BUCKETS + [self.MAX_BATCH]))

    def to_dict(self, redact: bool = True) -> Dict[str, Any]:
        d = {k: getattr(self, k) for k in self.field_names()}
        if redact and d.get("API_KEY"):
            d["API_KEY"] = "***"
        return d

    def model_yaml(self) -> Dict[str, Any]:
        """Per-model YAML overrides (``MODEL_CONFIG``), loaded with the safe loader."""
        if not self.MODEL_CONFIG:
            return {}
        import yaml

        with open(self.MODEL_CONFIG, "r", encoding="utf-8") as f:
            data = yaml.safe_load(f) or {}
        if not isinstance(data, dict):
            raise ValueError("MODEL_CONFIG must contain a mapping")
        return data
