import os, sys, time
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
import eigmi
ctx = eigmi.Context(0)
for sz in (4096, 262144, 524288, 2097152):
    h = np.ones(sz)
    keep = []
    t0 = time.perf_counter()
    for _ in range(10):
        keep.append(ctx.array(h))
    ctx.sync()
    t1 = time.perf_counter()
    del keep
    t2 = time.perf_counter()
    print(f"{sz*8/1e6:8.2f} MB: alloc+copy {1e3*(t1-t0)/10:.3f} ms each, free {1e3*(t2-t1)/10:.3f} ms each", flush=True)
