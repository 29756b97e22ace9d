# Inverse / shift-invert drivers at the reference's default size (src/dune-eigensolver.ini: ev.N = 200)
set -o pipefail
O=gpurun_out/inv200
mkdir -p $O
cat > $O/ref.ini <<'INI'
[grid]
N = 5
refine = 1
[islands]
scaling = 1.0
[mv]
N = 5
n_iter = 1000
m = 64
[ev]
N = 200
m =  4
maxiter = 4000
shift = 1e-3
regularization = 0.0
tol = 2e-3
verbose = 0
overlap = 3
method = raes
seed = 123
[parallel]
numthreads = 1
[mgs]
n = 20
m = 16
n_iter = 15
INI
timeout -k 10 300 dune-eigensolver_amd/bin/eigmi_harness -ini $O/ref.ini -run smallest > $O/smallest.log 2>&1 || exit 1
timeout -k 10 300 dune-eigensolver_amd/bin/eigmi_harness -ini $O/ref.ini -run largest > $O/largest.log 2>&1 || exit 1
EIGMI_INV_N=${INV_N:-200} timeout -k 10 400 python -u tools/bench_configs.py inv > $O/inv.jsonl 2> $O/inv.err || exit 1
