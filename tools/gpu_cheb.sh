set -o pipefail
mkdir -p gpurun_out/cheb
export SWEEP="${SWEEP:-EIGMI_EXP_PW=0;EIGMI_EXP_PW=128;EIGMI_EXP_PW=192;EIGMI_EXP_PW=256;EIGMI_EXP_PW=384;EIGMI_EXP_PW=512;EIGMI_EXP_PW=768;EIGMI_EXP_PW=256,EIGMI_EXP_NSEG=1;EIGMI_EXP_PW=512,EIGMI_EXP_NSEG=1}"
timeout -k 10 500 python -u tools/cheb_sweep.py --rounds 2 > gpurun_out/cheb/sweep.jsonl 2> gpurun_out/cheb/sweep.err
