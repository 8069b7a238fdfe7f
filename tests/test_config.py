"""Settings / .env loader (reference .env:1-3 + load_dotenv)."""
import pytest

from mlmicroservicetemplate_amd.config import Settings, load_dotenv, parse_dotenv


def test_parse_dotenv_features():
    text = """
# comment
NAME=example_model
PORT=5005
export SERVER_PORT=5000
QUOTED="a b # not comment"
SINGLE='$NAME literal'
INLINE=value # trailing comment
EXPANDED=${NAME}-x
DEFAULTED=${MISSING:-fallback}
MULTI="line1
line2"
EMPTY=
"""
    d = parse_dotenv(text)
    assert d["NAME"] == "example_model" and d["PORT"] == "5005" and d["SERVER_PORT"] == "5000"
    assert d["QUOTED"] == "a b # not comment"
    assert d["SINGLE"] == "$NAME literal"
    assert d["INLINE"] == "value"
    assert d["EXPANDED"] == "example_model-x"
    assert d["DEFAULTED"] == "fallback"
    assert d["MULTI"] == "line1\nline2"
    assert d["EMPTY"] == ""


def test_reference_env_defaults_and_precedence(tmp_path):
    env = tmp_path / ".env"
    env.write_text("NAME=example_model\nPORT=5005\nSERVER_PORT=5000\nMAX_BATCH=16\n")
    s = Settings.load(env_file=str(env), environ={"PORT": "6000"}, overrides={"MAX_BATCH": 64})
    assert s.NAME == "example_model"
    assert s.PORT == 6000  # environment beats .env
    assert s.SERVER_PORT == 5000
    assert s.MAX_BATCH == 64  # explicit override beats both
    assert s.GRAPH_BUCKETS[-1] >= 64


def test_types_and_lists():
    s = Settings.load(env_file=None, environ={"GRAPH_BUCKETS": "8,1,4", "REGISTER": "false", "CORS_ORIGINS": "http://a, http://b",
                                              "SERVER_PORT": "", "MAX_WAIT_US": "500"})
    assert s.GRAPH_BUCKETS == [1, 4, 8, 32]
    assert s.REGISTER is False
    assert s.CORS_ORIGINS == ["http://a", "http://b"]
    assert s.SERVER_PORT is None
    assert s.MAX_WAIT_US == 500


def test_api_key_file_and_redaction(tmp_path):
    kf = tmp_path / "key"
    kf.write_text("s3cret\n")
    s = Settings.load(env_file=None, environ={"API_KEY_FILE": str(kf)})
    assert s.API_KEY == "s3cret"
    assert s.to_dict()["API_KEY"] == "***"


def test_validation():
    with pytest.raises(ValueError):
        Settings.load(env_file=None, environ={"PORT": "70000"})
    with pytest.raises(ValueError):
        Settings.load(env_file=None, environ={"DTYPE": "int3"})


def test_load_dotenv_does_not_override(tmp_path):
    env = tmp_path / ".env"
    env.write_text("A=1\nB=2\n")
    environ = {"A": "0"}
    load_dotenv(str(env), environ=environ)
    assert environ == {"A": "0", "B": "2"}
    load_dotenv(str(env), override=True, environ=environ)
    assert environ["A"] == "1"


def test_repo_env_file_matches_reference():
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = Settings.load(env_file=os.path.join(root, ".env"), environ={})
    assert (s.NAME, s.PORT, s.SERVER_PORT) == ("example_model", 5005, 5000)
