"""Engine host staging (engine/staging.py + engine/csrc/staging.cpp): the native copy pool must
write exactly what the Python path writes, for any batch / sample size, under concurrent callers."""
import threading

import numpy as np
import pytest

from mlmicroservicetemplate_amd.engine import staging


@pytest.fixture(scope="module")
def native_ok():
    if staging._load() is None:
        pytest.fail(f"native staging module failed to build/load: {staging._mod_err}")
    return True


@pytest.mark.parametrize("threads", [0, 1, 3, 8])
@pytest.mark.parametrize("shape,n", [((224, 224, 3), 32), ((257,), 5), ((600_001,), 3), ((1,), 1)])
def test_native_gather_matches(native_ok, threads, shape, n):
    rng = np.random.default_rng(threads * 7 + n)
    st = staging.HostStager(threads, native=True)
    assert st.native
    samples = [rng.integers(0, 256, shape, dtype=np.uint8) for _ in range(n)]
    dst = np.full((n + 2, *shape), 7, np.uint8)
    for _ in range(3):
        st.gather(dst, samples)
        for i in range(n):
            np.testing.assert_array_equal(dst[i], samples[i])
        assert (dst[n:] == 7).all()  # rows past the batch untouched


def test_native_converts_dtype_and_layout(native_ok):
    st = staging.HostStager(2, native=True)
    dst = np.zeros((4, 6, 5), np.int32)
    base = np.arange(4 * 5 * 6, dtype=np.int64).reshape(4, 5, 6)
    samples = [base[i].T for i in range(4)]  # non-contiguous, other dtype
    st.gather(dst, samples)
    for i in range(4):
        np.testing.assert_array_equal(dst[i], samples[i].astype(np.int32))


def test_native_rejects_wrong_size(native_ok):
    st = staging.HostStager(2, native=True)
    dst = np.zeros((2, 10), np.uint8)
    with pytest.raises(ValueError):
        st.gather(dst, [np.zeros(10, np.uint8), np.zeros(11, np.uint8)])


def test_native_concurrent_callers(native_ok):
    """Two threads share one stager (two engines' submitters): batches never mix."""
    st = staging.HostStager(3, native=True)
    errors = []

    def run(seed):
        rng = np.random.default_rng(seed)
        dst = np.zeros((16, 40_000), np.uint8)
        try:
            for _ in range(60):
                samples = [rng.integers(0, 256, 40_000, dtype=np.uint8) for _ in range(16)]
                st.gather(dst, samples)
                for i in range(16):
                    if not np.array_equal(dst[i], samples[i]):
                        errors.append((seed, i))
                        return
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=run, args=(s,)) for s in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def test_python_fallback_matches():
    rng = np.random.default_rng(1)
    st = staging.HostStager(4, native=False)
    assert not st.native
    samples = [rng.integers(0, 256, (32, 32, 3), dtype=np.uint8) for _ in range(12)]
    dst = np.zeros((12, 32, 32, 3), np.uint8)
    st.gather(dst, samples)
    for i in range(12):
        np.testing.assert_array_equal(dst[i], samples[i])
