#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy from hipcc's kernel-resource-usage remarks.

    python tools/resource_usage.py csrc/k_spmv.hip [name-regex]
(compiles the device code of one source for gfx950 into /tmp; prints one line per kernel)"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-I../include",
       "--offload-arch=gfx950", "-munsafe-fp-atomics", "--cuda-device-only", "-c", src, "-o", "/tmp/ru_dev.o",
       "-Rpass-analysis=kernel-resource-usage"]
err = subprocess.run(cmd, cwd="/root/repo/dune-eigensolver_amd", capture_output=True, text=True).stderr
cur, row = None, {}
rows = []
for line in err.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        if cur:
            rows.append((cur, row))
        cur, row = m.group(1), {}
        continue
    m = re.search(r"remark:\s+([^:]+): (\S+)", line)
    if cur and m:
        row[m.group(1).strip()] = m.group(2)
if cur:
    rows.append((cur, row))
for name, r in rows:
    dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    if pat and not pat.search(dn):
        continue
    print(f"{dn[:110]:110s} vgpr {r.get('VGPRs', '?'):>4s} agpr {r.get('AGPRs', '?'):>3s} "
          f"sgpr {r.get('SGPRs', '?'):>3s} scratch {r.get('ScratchSize [bytes/lane]', '?'):>4s} "
          f"occ {r.get('Occupancy [waves/SIMD]', '?')}")
