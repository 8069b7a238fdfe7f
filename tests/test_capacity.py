"""Auto batch planning (MAX_BATCH=0, scheduler/capacity.py): HBM / SLO / cap bounds."""
from mlmicroservicetemplate_amd.config import Settings
from mlmicroservicetemplate_amd.scheduler.capacity import buckets_up_to, plan_batch, pow2_floor


def test_pow2_and_buckets():
    assert pow2_floor(1) == 1 and pow2_floor(33) == 32 and pow2_floor(64) == 64
    assert buckets_up_to(32) == [1, 2, 4, 8, 16, 32]
    assert buckets_up_to(1) == [1]


def test_slo_bound():
    # 288 GB free, 10 MB/sample, 5 slots -> HBM allows ~5000; 0.02 ms/sample + 0.5 ms fixed in a 3 ms SLO -> 125 -> 64
    p = plan_batch(10e6, 288e9, 0.9, 5, 0.02, 0.5, 3.0, 1024)
    assert p.limit == "slo" and p.max_batch == 64


def test_hbm_bound_and_cap():
    p = plan_batch(2e9, 40e9, 0.5, 2, 0.001, 0.0, 1000.0, 1024)  # 0.5*40e9/(2*2e9) = 5 -> 4
    assert p.limit == "hbm" and p.max_batch == 4
    p = plan_batch(1e6, 288e9, 0.9, 5, 0.0001, 0.0, 1000.0, 256)
    assert p.limit == "cap" and p.max_batch == 256
    p = plan_batch(1e12, 1e9, 0.9, 5, 1.0, 0.0, 0.5, 256)  # nothing fits: still 1
    assert p.max_batch == 1


def test_settings_accept_auto():
    s = Settings.load(env_file=None, environ={}, overrides={"MAX_BATCH": 0})
    assert s.MAX_BATCH == 0 and s.LATENCY_SLO_MS > 0 and s.MAX_BATCH_CAP >= 1
