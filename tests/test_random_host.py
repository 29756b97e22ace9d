"""The drivers' start vectors (eigensolver.hh:50-55: std::mt19937{seed} + std::normal_distribution
<double>{0, 1}) come from the library's own polar-method walk with libstdc++'s constants folded
(api.cpp host_random_normal); bar: BITWISE the oracle's draws, which call the std:: objects
themselves (oracle.cc orc_random_vec / orc_random_mv8), for odd and even counts and several seeds.
Host only: no device."""
import time

import numpy as np
import pytest

import eigmi
import oracle


@pytest.mark.parametrize("seed", [123, 0, 5, 11, 4294967295])
@pytest.mark.parametrize("count", [0, 1, 2, 7, 4096 * 8 + 1, 100003])
def test_random_normal_bitwise_std(seed, count):
    a = eigmi.random_normal(count, seed)
    b = oracle.random_vec(count, seed) if count else np.zeros(0)
    assert a.dtype == b.dtype and a.shape == b.shape
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))


def test_random_normal_matches_block_fill_and_is_faster():
    n, m = 4096, 8
    a = eigmi.random_normal(n * m, 123)
    assert np.array_equal(a.view(np.uint64), oracle.random_mv8(n, m, 123).view(np.uint64))
    t0 = time.perf_counter()
    for _ in range(5):
        eigmi.random_normal(n * m, 123)
    t_lib = (time.perf_counter() - t0) / 5
    t0 = time.perf_counter()
    for _ in range(5):
        oracle.random_mv8(n, m, 123)
    t_std = (time.perf_counter() - t0) / 5
    print(f"32768 variates: library {t_lib * 1e3:.3f} ms, std:: objects {t_std * 1e3:.3f} ms")
