"""Matrix Market import / export (eig_mm_read / eig_mm_write) -- the wire format
DUNE writes with Dune::storeMatrixMarket.  Checked against scipy.io (the independent reader /
writer): general and symmetric files, pattern files, duplicates, 3x3 block grouping; on the GPU
an imported matrix multiplies bitwise like the generator's."""
import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp

import eigmi
import oracle


def as_scipy(rp, c, v, ncols, br=1):
    if br == 1:
        return sp.csr_matrix((v, c, rp), shape=(rp.size - 1, ncols))
    return sp.bsr_matrix((v.reshape(-1, br, br), c, rp), shape=((rp.size - 1) * br, ncols * br)).tocsr()


def test_read_general_and_symmetric(tmp_path):
    A = oracle.laplace2d(9).to_scipy()
    for sym in ("general", "symmetric"):
        p = tmp_path / f"a_{sym}.mtx"
        scipy.io.mmwrite(str(p), A, symmetry=sym)
        rp, c, v, nc = eigmi.mm_read(str(p))
        B = as_scipy(rp, c, v, nc)
        assert nc == A.shape[1] and abs(B - A).max() == 0
        assert all(np.all(np.diff(c[rp[i]:rp[i + 1]]) > 0) for i in range(rp.size - 1))


def test_read_pattern_and_duplicates(tmp_path):
    p = tmp_path / "dup.mtx"
    p.write_text("%%MatrixMarket matrix coordinate real general\n% comment\n3 4 4\n1 2 1.5\n1 2 2.0\n3 4 -1\n2 1 7\n")
    rp, c, v, nc = eigmi.mm_read(str(p))
    assert nc == 4 and list(rp) == [0, 1, 2, 3] and list(c) == [1, 0, 3] and list(v) == [3.5, 7.0, -1.0]
    q = tmp_path / "pat.mtx"
    q.write_text("%%MatrixMarket matrix coordinate pattern symmetric\n2 2 2\n1 1\n2 1\n")
    rp, c, v, nc = eigmi.mm_read(str(q))
    assert list(rp) == [0, 2, 3] and list(c) == [0, 1, 0] and list(v) == [1.0, 1.0, 1.0]


def test_blocked_roundtrip(tmp_path):
    Q = oracle.q1elast(3)
    p = tmp_path / "q1.mtx"
    eigmi.mm_write(str(p), Q.rowptr, Q.col, Q.val, br=3, bc=3)
    ref = Q.to_scipy().tocsr()
    got = scipy.io.mmread(str(p)).tocsr()
    assert abs(got - ref).max() == 0  # %.17g round trips exactly
    rp, c, v, nc = eigmi.mm_read(str(p), br=3)
    assert np.array_equal(rp, Q.rowptr) and np.array_equal(c, Q.col) and np.array_equal(v, Q.val)
    s = tmp_path / "q1s.mtx"
    eigmi.mm_write(str(s), Q.rowptr, Q.col, Q.val, br=3, bc=3, symmetric=True)
    assert abs(scipy.io.mmread(str(s)).tocsr() - ref).max() == 0


def test_errors(tmp_path):
    p = tmp_path / "bad.mtx"
    p.write_text("%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n")
    with pytest.raises(eigmi.EigError):
        eigmi.mm_read(str(p))
    q = tmp_path / "odd.mtx"
    q.write_text("%%MatrixMarket matrix coordinate real general\n4 4 1\n1 1 1\n")
    with pytest.raises(eigmi.EigError):
        eigmi.mm_read(str(q), br=3)  # 4 rows are not 3x3 blocks
    with pytest.raises(eigmi.EigError):
        eigmi.mm_read(str(tmp_path / "missing.mtx"))


@pytest.mark.gpu
def test_imported_matrix_on_gpu(ctx, tmp_path):
    A = oracle.poisson3d(12)
    p = tmp_path / "p.mtx"
    scipy.io.mmwrite(str(p), A.to_scipy(), symmetry="symmetric")
    rp, c, v, nc = eigmi.mm_read(str(p))
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v)
    x = np.random.default_rng(3).standard_normal(A.n)
    assert np.array_equal(M.mv_host(x), oracle.csr_mv(A, x))
