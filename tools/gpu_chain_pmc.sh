# Stall counters of the block-inverse chain (k_binv_chain) at 200^2 (tools/time_apply.py)
set -o pipefail
O=gpurun_out/chainpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD --output-format csv -d $O/p1 -o pmc -- python3 -u tools/time_apply.py 200 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA --output-format csv -d $O/p2 -o pmc -- python3 -u tools/time_apply.py 200 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
python3 tools/pmc_summary.py $O/p1 $O/p2 --match binv_chain
