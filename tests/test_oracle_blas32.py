"""The float32 arithmetic of utils.py:10-11 restated operation by operation
(oracle.blas32_*: numpy 2.2's einsum row norms, sklearn's division, OpenBLAS
0.3.29 SkylakeX sgemm's small-matrix and K-blocked summation orders) equals
numpy/sklearn bit for bit in this container, for the group shapes the
reference's per-(round, bucket) products take -- and on the r5 fixtures'
float32 inputs.  The GPU split mode computes the same values
(test_gpu_split_mode.py); this pins the restatement to the reference's own
libraries (parity anchored on the reference's dependencies: numpy, OpenBLAS)."""
import numpy as np
import pytest

import lmi_oracle as O


def _blas_is_skylakex():
    import glob
    import os
    import ctypes
    libs = glob.glob(os.path.join(os.path.dirname(np.__file__), "..", "numpy.libs", "*openblas*"))
    for p in libs:
        try:
            f = getattr(ctypes.CDLL(p), "scipy_openblas_get_corename64_")
            f.restype = ctypes.c_char_p
            return f().decode()
        except (OSError, AttributeError):
            continue
    return None


pytestmark = pytest.mark.skipif(_blas_is_skylakex() != "SkylakeX",
                                reason="the restated orders are OpenBLAS's SkylakeX kernels")


@pytest.mark.parametrize("M,N", [(2, 4), (4, 2), (5, 17), (13, 80), (16, 75), (4, 300), (5, 241),
                                 (100, 40), (24, 64), (40, 200), (25, 14), (6, 7), (13, 22), (7, 30),
                                 (15, 9), (31, 37)])
def test_blas32_pairwise_cosine_is_numpys(M, N):
    rng = np.random.default_rng(M * 1000 + N)
    x = (rng.standard_normal((M, 768)) * 0.05 + 0.01).astype(np.float32)
    y = (rng.standard_normal((N, 768)) * 0.05).astype(np.float32)
    got = O.blas32_pairwise_cosine(x, y)
    assert got is not None and got.dtype == np.float32
    np.testing.assert_array_equal(got, O.pairwise_cosine(x, y))


def test_blas32_kernel_boundary():
    assert O.blas32_kernel(4, 300, 768) == "small"     # 921,600 = 96 * 96 * 100
    assert O.blas32_kernel(4, 301, 768) == "blocked"
    assert O.blas32_kernel(1, 50, 768) is None           # gemv
    assert O.blas32_kernel(3, 3, 768) is None            # tiny


def test_blas32_random_small_shapes():
    """Sixty random shapes of the small-matrix kernel (every corner block
    remainder): all bit for bit."""
    rng = np.random.default_rng(5)
    n = 0
    while n < 60:
        M, N = int(rng.integers(2, 40)), int(rng.integers(2, 60))
        if O.blas32_kernel(M, N, 768) != "small":
            continue
        x = rng.standard_normal((M, 768)).astype(np.float32)
        y = rng.standard_normal((N, 768)).astype(np.float32)
        np.testing.assert_array_equal(O.blas32_pairwise_cosine(x, y), O.pairwise_cosine(x, y))
        n += 1


def test_blas32_on_the_r5_fixture_groups():
    """Every (round, bucket) group of the r5 float32 search fixtures whose
    shape is restated: the restatement's distances equal the oracle's (=
    numpy's, which equal the reference's: test_oracle_golden_r5)."""
    from test_oracle_golden_r5 import CASES, G5, inputs_r5
    checked = 0
    for name, c in CASES.items():
        _, n, nq, C, R, k, mode, arch, seed, thr, qdt = c
        w, x, q, arith = inputs_r5(name)
        if arith != "f32":
            continue
        classes = G5[f"search_{name}__classes"].astype(np.int64)
        order, off = O.layout(w["labels"], C)
        for r in range(R):
            for cat in np.unique(classes[:, r]):
                G = np.nonzero(classes[:, r] == cat)[0]
                y = x[order[off[cat]:off[cat + 1]]]
                got = O.blas32_pairwise_cosine(q[G], y)
                if got is None:
                    continue
                np.testing.assert_array_equal(got, O.pairwise_cosine(q[G], y))
                checked += 1
    assert checked > 20
