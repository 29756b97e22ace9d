import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd")); sys.path.insert(0, ROOT)
import eigmi, oracle
ctx = eigmi.Context(0)
for N in (24, 40, 64):
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, N)
    rp, c, v = eigmi.scrambled_rcm(rp, c, v, 123)
    A = oracle.CSR(rp.size - 1, rp, c, v)
    ra, rb = oracle.lanczos_fused(A, oracle.random_vec(A.n, 123), 10)
    for flags in (0, eigmi.MAT_NO_BAND, eigmi.MAT_NO_STENCIL):
        M = eigmi.Matrix.from_bcsr(ctx, rp, c, v, flags=flags)
        for cpf in (0, 1):
            M.tune(sell_cpf=cpf)
            a, b, _ = eigmi.lanczos_run(M, 10, seed=123, fused=True)
            print(N, flags, "stencil", M.info.stencil_slices, "/", M.info.nslices, "cpf", cpf, "maxrel", float(np.max(np.abs(a - ra) / np.abs(ra))), flush=True)
        M.close()
