"""bert plugin's native-front-end contract on CPU: packed row layout (ids | type ids | length at
the largest seq bucket) equals the Python path's pack_requests, and raw client bodies are never
accepted as rows (``raw_samples`` False)."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from mlmicroservicetemplate_amd.api.multipart import Part
from mlmicroservicetemplate_amd.models import bert
from mlmicroservicetemplate_amd.plugins.text_classifier import BertPlugin


def _plugin(max_seq):  # geometry set by hand (configure() is tested below)
    p = BertPlugin()
    p.max_seq = max_seq
    p.tokenizer = bert.HashTokenizer(30522)
    return p


def test_native_row_matches_pack_requests(monkeypatch):
    monkeypatch.setenv("MLS_NATIVE_TOKENIZER", "0")
    p = _plugin(128)
    spec = p.native_spec()
    assert spec == {"sample_bytes": (2 * 128 + 1) * 4, "result": "topk", "raw_samples": False}
    for text in ["hello world", "word " * 300, ""]:
        part = Part(name="text", data=text.encode())
        row = p.native_preprocess(part)
        assert row.dtype == np.int32 and row.nbytes == spec["sample_bytes"]
        want = bert.pack_requests([p.preprocess(part)], 128).numpy()[0]
        np.testing.assert_array_equal(row, want)


def test_native_tokenizer_default_on_and_opt_out(monkeypatch):
    monkeypatch.delenv("MLS_NATIVE_TOKENIZER", raising=False)
    assert _plugin(128).native_spec()["text_hash"] == [30522, 128, 128, bert.CLS_ID, bert.SEP_ID]
    monkeypatch.setenv("MLS_NATIVE_TOKENIZER", "0")
    assert "text_hash" not in _plugin(128).native_spec()


def test_native_seq_is_largest_bucket_below_max_seq():
    p = _plugin(100)  # buckets 32, 64 fit: rows are packed at 64, longer texts truncated like the Python path
    row = p.native_preprocess(Part(name="text", data=("w " * 200).encode()))
    assert row.shape == (2 * 64 + 1,) and row[-1] == 64


ASCII = "".join(chr(i) for i in range(128))


@settings(max_examples=300, deadline=None)
@given(st.text(alphabet=ASCII, max_size=400), st.sampled_from([(128, 128), (100, 64), (16, 16)]))
def test_cpp_hash_tokenizer_matches_python(text, lens):
    """The C++ tokenizer on the native front end's I/O threads == HashTokenizer (+ the row cut)."""
    from mlmicroservicetemplate_amd.frontend.native import load_extension

    max_len, seq = lens
    ext = load_extension()
    want = bert.HashTokenizer(30522).encode(text, max_len)[:seq]
    assert ext.hash_tokenize(text, 30522, max_len, seq) == want


def test_cpp_hash_tokenizer_defers_non_ascii():
    from mlmicroservicetemplate_amd.frontend.native import load_extension

    assert load_extension().hash_tokenize("caf\u00e9 na\u00efve", 30522, 128, 128) is None


def _settings(tmp_path, max_seq):
    from mlmicroservicetemplate_amd.config import Settings

    cfg = tmp_path / "bert.yaml"
    cfg.write_text(f"max_seq: {max_seq}\nnum_labels: 3\n")
    return Settings.load(env_file=None, environ={}, overrides={
        "MODEL": "bert", "REGISTER": False, "MODEL_CONFIG": str(cfg), "IO_THREADS": 1})


@pytest.mark.parametrize("max_seq,seq", [(64, 64), (256, 256), (100, 64)])
def test_native_service_spec_follows_model_config(tmp_path, monkeypatch, max_seq, seq):
    """The spec NativeService builds its C++ Server from is derived from MODEL_CONFIG before
    init() runs: rows the decode threads pack have exactly the Server's sample size, and the
    opt-in C++ tokenizer is actually handed to the Server (native_spec ran before
    init and saw max_seq=128 and no tokenizer)."""
    from mlmicroservicetemplate_amd.frontend.native import NativeService
    from mlmicroservicetemplate_amd.plugins.base import PluginContext

    monkeypatch.setenv("MLS_NATIVE_TOKENIZER", "1")
    s = _settings(tmp_path, max_seq)
    p = BertPlugin()
    svc = NativeService(s, p, PluginContext(settings=s), host="127.0.0.1", port=0)
    try:
        assert svc.spec["sample_bytes"] == (2 * seq + 1) * 4
        assert svc.spec["text_hash"] == [30522, max_seq, seq, bert.CLS_ID, bert.SEP_ID]
        assert p.labels == ["label_0", "label_1", "label_2"]
        row = p.native_preprocess(Part(name="text", data=("w " * 400).encode()))
        assert row.nbytes == svc.spec["sample_bytes"] and row[-1] == seq
    finally:
        svc.srv.stop()


def test_native_spec_requires_configure():
    with pytest.raises(RuntimeError):
        BertPlugin().native_spec()
