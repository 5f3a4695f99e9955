#!/bin/bash
# PMC counters of the in-step training GEMM (stream-K weight-gradient GEMM + flash attention) over 2 bench steps,
# one rocprofv3 run per counter pass (per-block limits: 8 SQ, 4 TCC, 2 TA, 2 GRBM).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_sk_fa_r3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "gemm_sk|fa64" --output-format csv -d $O -o p$i -- python3 $R/bench.py --mode spmd --steps 2 --warmup 1 > $O/log$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $O/log$i.txt; exit 1; }
  echo "pass $i ok"
done
python3 $R/tools/prof_summarize.py $O > $O/summary.txt && cat $O/summary.txt
