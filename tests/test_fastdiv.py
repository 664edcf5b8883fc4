"""Host-side exhaustive checks of the two integer-division shortcuts the gfx950 kernels use in
place of a ~40-100 instruction integer `/`:

* ``fdiv`` (kernels/convn.hip, bwd mode 5 epilogue): q = trunc(float(x) * (1.f / d)) plus one
  correction step, valid for 0 <= x < 2^24;
* ``FastDiv`` (kernels/common.h, the stem pool kernels' index maps): the Granlund-Montgomery
  round-up multiply, q = (umulhi(x, m) + x) >> s, valid for 0 <= x < 2^31.

Both are emulated bit-exactly with numpy (IEEE float32 multiply and reciprocal, round-to-nearest;
float -> int truncation; 32-bit unsigned umulhi) and compared with integer division for every x
in range for the divisors the ResNet shapes use. CPU only (no GPU needed).
"""
import numpy as np
import pytest

# Ho*Wo and Wo of every ResNet-50 / WRN output grid at 224^2 (and the test shapes' grids)
DIVISORS = [3136, 56, 784, 28, 196, 14, 49, 7, 12544, 112, 64, 8, 6, 3, 2, 1, 4, 16, 32, 100, 10, 144, 12]


def fdiv_emul(x: np.ndarray, d: int) -> np.ndarray:
    inv = np.float32(1.0) / np.float32(d)
    q = (x.astype(np.float32) * inv).astype(np.int64)  # v_cvt_i32_f32 truncates
    r = x - q * d
    return q + (r >= d).astype(np.int64) - (r < 0).astype(np.int64)


def fastdiv_params(d: int):
    s = 0
    while (1 << s) < d:
        s += 1
    m = ((1 << 32) * ((1 << s) - d)) // d + 1
    assert 0 < m < (1 << 32)
    return m, s


def fastdiv_emul(x: np.ndarray, d: int) -> np.ndarray:
    m, s = fastdiv_params(d)
    hi = (x.astype(np.uint64) * np.uint64(m)) >> np.uint64(32)
    return ((hi + x.astype(np.uint64)) >> np.uint64(s)).astype(np.int64)


@pytest.mark.parametrize("d", DIVISORS)
def test_fdiv_float_reciprocal_exhaustive_below_2_24(d):
    for lo in range(0, 1 << 24, 1 << 22):
        x = np.arange(lo, lo + (1 << 22), dtype=np.int64)
        np.testing.assert_array_equal(fdiv_emul(x, d), x // d)


@pytest.mark.parametrize("d", DIVISORS + [(1 << 31) - 1, (1 << 30) + 7, 65537, 1000003])
def test_fastdiv_magic_multiply(d):
    # exhaustive below 2^24, then the top of the range and every multiple boundary sampled
    for lo in range(0, 1 << 24, 1 << 22):
        x = np.arange(lo, lo + (1 << 22), dtype=np.int64)
        np.testing.assert_array_equal(fastdiv_emul(x, d), x // d)
    rng = np.random.default_rng(d)
    top = np.concatenate([np.arange((1 << 31) - 4096, 1 << 31, dtype=np.int64),
                          rng.integers(0, 1 << 31, 1 << 20, dtype=np.int64)])
    ks = np.arange(1, min((1 << 31) // d, 1 << 20), dtype=np.int64)
    edges = np.concatenate([ks * d - 1, ks * d])
    for x in (top, edges[edges < (1 << 31)]):
        np.testing.assert_array_equal(fastdiv_emul(x, d), x // d)
