#!/usr/bin/env python3
"""One StandardLargest solve at C2 (3-D Poisson 128^3, nev 8, 40 iterations, tol 0) for a kernel
trace: `rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o sl -- python3 tools/sl_trace.py`
shows the per-iteration kernels of the driver (MGS look-ahead read + write pass, the fused SpMM +
diagonal dots) and the gaps between them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
import eigmi  # noqa: E402

N = int(os.environ.get("EIGMI_SL_N", "128"))
ctx = eigmi.Context(0)
rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, N)
M = eigmi.Matrix.from_bcsr(ctx, rp, c, v, flags=eigmi.MAT_NO_UNIFORM)
ev, _, it = eigmi.standard_largest(M, 0.0, 0.0, 41, 8, 123, want_evec=False)
print(f"N {N}: {it} iterations, spmm8 kernel {M.kernel('spmm8')}, ritz0 {ev[0]!r}")
M.close()
ctx.close()
