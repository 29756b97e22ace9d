"""ARPACK driving the GPU operator: the reference's ArpackMLGeneo wrapper hands ARPACK's reverse
communication a `multMv` that calls BCRSMatrix::mv (arpack_geneo_wrapper.hh:269-279); the drop-in
replaces that mv with eig_mv (include/eigmi.hh).  ARPACK itself is ARPACK-NG as
bundled by scipy (scipy.sparse.linalg.eigsh).

Bar: ARPACK with the GPU mv and ARPACK with the restated reference mv (oracle.csr_mv / bcsr_mv, the
BCRSMatrix::mv row loop) see bitwise the same operator, so the whole reverse-communication trajectory
is the same: eigenvalues and eigenvectors BITWISE equal -- on the C3 operator (3-D Q1 elasticity,
BCRSMatrix<FieldMatrix<double,3,3>>) and on the 3-D Poisson band image.  Against ARPACK on scipy's
own CSR matvec (other rounding) within 1e-10 relative."""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as ssl

import eigmi
import oracle

pytestmark = pytest.mark.gpu


def _scipy(A):
    return sp.csr_matrix(A.to_scipy())


def _eigsh(op, n, k, which):
    return ssl.eigsh(op, k=k, which=which, v0=np.ones(n), tol=1e-12, ncv=4 * k + 1, maxiter=5000)


@pytest.mark.parametrize("name,make,k,which", [
    ("q1elast16_3x3", lambda: oracle.q1elast(16), 6, "LA"),
    ("poisson3d_24", lambda: oracle.poisson3d(24), 5, "LA"),
    ("q1elast12_3x3_smallest", lambda: oracle.q1elast(12), 4, "SA"),
])
def test_arpack_with_gpu_mv(ctx, name, make, k, which):
    A = make()
    n = A.nrows * A.br
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val, A.br, A.bc)
    calls = [0]

    def gpu_mv(x):
        calls[0] += 1
        return M.mv_host(np.asarray(x, np.float64).ravel())

    w_gpu, v_gpu = _eigsh(ssl.LinearOperator((n, n), matvec=gpu_mv, dtype=np.float64), n, k, which)
    w_ref, v_ref = _eigsh(ssl.LinearOperator((n, n), matvec=lambda x: oracle.csr_mv(A, np.ravel(x)),
                                              dtype=np.float64), n, k, which)
    w_sp, _ = _eigsh(_scipy(A), n, k, which)
    M.close()
    print(f"{name}: n = {n}, {calls[0]} GPU mv calls, eigenvalues {np.round(w_gpu, 10)}, "
          f"max rel vs scipy CSR {np.max(np.abs(w_gpu - w_sp) / np.abs(w_sp)):.1e}")
    assert np.array_equal(w_gpu, w_ref) and np.array_equal(v_gpu, v_ref)
    assert np.allclose(w_gpu, w_sp, rtol=1e-10, atol=0)
    # and they are eigenpairs of the operator
    S = _scipy(A)
    r = np.linalg.norm(S @ v_gpu - v_gpu * w_gpu, axis=0) / np.abs(w_gpu)
    assert r.max() < 1e-8
