set -o pipefail
mkdir -p gpurun_out/cheb
export SWEEP="${SWEEP:-EIGMI_EXP_NBW=1;EIGMI_EXP_NBW=4;EIGMI_EXP_NBW=4,EIGMI_EXP_NSEG=1;EIGMI_EXP_NBW=1,EIGMI_EXP_NSEG=1;EIGMI_EXP_NBW=4,EIGMI_EXP_NSEG=4}"
timeout -k 10 400 python -u tools/cheb_sweep.py > gpurun_out/cheb/sweep.jsonl 2> gpurun_out/cheb/sweep.err
