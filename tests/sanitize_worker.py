"""Exercised by tests/test_sanitize.py under the clang ASan/UBSan runtime (EIGMI_LIB_VARIANT=san):
the host code paths of libeigmi that need no device -- envelope LU, Matrix Market I/O, reordering,
generators, the distributed plan functions, argument errors."""
import os
import sys
import tempfile

import numpy as np

import eigmi
import oracle

assert eigmi.LIB_PATH.endswith("libeigmi_san.so"), eigmi.LIB_PATH
for A in (oracle.poisson3d(8), oracle.laplace2d(20), oracle.laplace2d(12, "pu", 3)):
    if A.br == 1:
        B = oracle.CSR(A.nrows, A.rowptr, A.col, A.val.copy())
        B.val[B.col == np.repeat(np.arange(B.n), np.diff(B.rowptr))] += 0.5
        d = eigmi.LU.from_bcsr(None, B.rowptr, B.col, B.val).export()
        assert d["Lp"][-1] > 0
Q = oracle.q1elast(3)
d = eigmi.LU.from_bcsr(None, Q.rowptr, Q.col, Q.val, br=3).export()
with tempfile.TemporaryDirectory() as td:
    for A in (oracle.laplace2d(10), oracle.q1elast(2)):
        p = os.path.join(td, "a.mtx")
        eigmi.mm_write(p, A.rowptr, A.col, A.val, br=A.br, bc=A.bc)
        rp, c, v = eigmi.mm_read(p, br=A.br)[:3]
        assert np.array_equal(rp, A.rowptr) and np.array_equal(c, A.col) and np.array_equal(v, A.val)
A = oracle.poisson3d(10)
rp, c, v = eigmi.scrambled_rcm(A.rowptr, A.col, A.val, 5)
assert rp[-1] == A.rowptr[-1]
for kind in range(8):
    eigmi.gen_matrix(kind, 6)
    eigmi.gen_rows(kind, 6, 10, 20)
P = 3
n = 12 ** 3
parts = [eigmi.row_partition(n, P, r, align=144) for r in range(P)]
ranks = []
for r, (b, cnt) in enumerate(parts):
    rp, c, v = eigmi.gen_rows(eigmi.GEN_POISSON3D, 12, b, cnt)
    w = eigmi.plan_window(b, cnt, rp, c)
    ranks += [b, cnt, w[3], w[4]]
for r in range(P):
    eigmi.plan_halo(P, r, np.array(ranks, np.int64), eigmi.plan_window(*parts[r], *eigmi.gen_rows(
        eigmi.GEN_POISSON3D, 12, *parts[r])[:2])[0])
for bad in (lambda: eigmi.reorder_rcm(np.array([0, 1], np.int64), np.array([7], np.int32)),
            lambda: eigmi.LU.from_bcsr(None, np.array([0, 1], np.int64), np.array([0], np.int32), np.array([0.0]))):
    try:
        bad()
        raise SystemExit("expected an error")
    except eigmi.EigError:
        pass
print("sanitize worker ok")
sys.stdout.flush()
