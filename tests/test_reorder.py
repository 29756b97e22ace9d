"""Host reordering utilities (eig_reorder_rcm, eig_permute_symmetric; reorder.cpp): permutation
validity, B = P A P^T against scipy, and the RCM bandwidth against scipy's own RCM."""
import numpy as np
import pytest

import eigmi
import oracle


def _sp(A):
    import scipy.sparse as sp
    return sp.csr_matrix((A.val, A.col, A.rowptr), shape=(A.n, A.n))


@pytest.mark.parametrize("mk", [lambda: oracle.poisson3d(12), lambda: oracle.laplace2d(40),
                                lambda: oracle.laplace2d(20, "pu", 3)])
def test_permute_symmetric_matches_scipy(mk):
    A = mk()
    p = np.random.default_rng(3).permutation(A.n).astype(np.int64)
    rp, c, v = eigmi.permute_symmetric(A.rowptr, A.col, A.val, p)
    S = _sp(A)[p][:, p].tocsr()
    S.sort_indices()
    assert np.array_equal(rp, S.indptr) and np.array_equal(c, S.indices) and np.array_equal(v, S.data)
    assert all(np.all(np.diff(c[rp[i]:rp[i + 1]]) > 0) for i in range(0, A.n, 97))


def test_rcm_bandwidth():
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    A = oracle.poisson3d(20)
    p0 = np.random.default_rng(5).permutation(A.n).astype(np.int64)
    rp, c, v = eigmi.permute_symmetric(A.rowptr, A.col, A.val, p0)
    perm = eigmi.reorder_rcm(rp, c)
    assert np.array_equal(np.sort(perm), np.arange(A.n))
    r2, c2, _ = eigmi.permute_symmetric(rp, c, v, perm)
    rows = np.repeat(np.arange(A.n), np.diff(r2))
    bw = np.abs(c2 - rows).max()
    import scipy.sparse as sp
    S = sp.csr_matrix((v, c, rp), shape=(A.n, A.n))
    q = reverse_cuthill_mckee(S, symmetric_mode=True)
    T = S[q][:, q].tocoo()
    bw_scipy = np.abs(T.row - T.col).max()
    assert bw < 400 * 3 and bw <= 1.25 * bw_scipy, (bw, bw_scipy)


def test_reorder_errors():
    rp = np.array([0, 1, 2], np.int64)
    with pytest.raises(eigmi.EigError):
        eigmi.reorder_rcm(rp, np.array([0, 5], np.int32))
    with pytest.raises(eigmi.EigError):
        eigmi.permute_symmetric(rp, np.array([0, 1], np.int32), np.ones(2), np.array([0, 0], np.int64))


def test_scrambled_rcm_keeps_spectrum():
    A = oracle.poisson3d(6)
    rp, c, v = eigmi.scrambled_rcm(A.rowptr, A.col, A.val, 9)
    B = oracle.CSR(A.n, rp, c, v)
    ea = np.linalg.eigvalsh(_sp(A).toarray())
    eb = np.linalg.eigvalsh(_sp(B).toarray())
    assert np.allclose(ea, eb, rtol=0, atol=1e-12)
