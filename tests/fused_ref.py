"""Reference pieces for the guarded fused Lanczos step's tests (CPU oracle only): shifted
operators, the classic two-reduction recurrence (orc_lanczos_rotating), and its own run-to-run
spread, against which the fused step is judged."""
import numpy as np

import oracle


def shifted(A, sigma, rows=None, add=0.0):
    """A + sigma I (every diagonal entry stored here), plus `add` on the diagonal of `rows`."""
    v = A.val.copy()
    rows = set(rows or ())
    for i in range(A.n):
        for p in range(A.rowptr[i], A.rowptr[i + 1]):
            if A.col[p] == i:
                v[p] += sigma + (add if i in rows else 0.0)
    return oracle.CSR(A.n, A.rowptr, A.col, v)


def classic(A, u0, k):
    """The two-reduction recurrence over three rotating vectors (orc_lanczos_rotating)."""
    u0 = np.array(u0, dtype=np.float64)
    u1, u2 = np.zeros(A.n), np.zeros(A.n)
    a, b = np.zeros(k), np.zeros(k + 1)
    oracle.lib.orc_lanczos_rotating(A.n, A.rowptr, A.col, A.val, k, u0, u1, u2, a, b)
    return a, b


def classic_spread(A, u0, k, cb):
    """The classic recurrence's own run-to-run spread: max relative beta change when u0 is
    perturbed at 1e-16 / 1e-15 (two seeds).  Lanczos without re-orthogonalisation amplifies the
    rounding of each step once Ritz values converge, and the rounding is eps ||A + sigma I||, so
    at A + 1e6 I (beta ~ 3) two classic runs already differ by ~6e-10 after 60 steps."""
    out = 0.0
    for seed, eps in ((1, 1e-16), (2, 1e-15)):
        _, pb = classic(A, u0 * (1 + eps * np.random.default_rng(seed).standard_normal(A.n)), k)
        out = max(out, float(np.max(np.abs(pb - cb) / np.abs(cb))))
    return out


def top_ritz(a, b):
    return np.linalg.eigvalsh(np.diag(a) + np.diag(b[1:-1], 1) + np.diag(b[1:-1], -1))[-1]
