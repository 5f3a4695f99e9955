#!/bin/bash
# Round 6: step kernel profile + per-GEMM PMC passes (MFMA util, L2, LDS), SPMD mode.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/step_r6b
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o run -- python3 $R/bench.py --mode spmd --steps 6 --warmup 2 > $O/step_bench.log 2>&1 || { echo "step prof failed"; tail -20 $O/step_bench.log; exit 1; }
grep -o '"value": [0-9.]*' $O/step_bench.log
python3 $R/tools/prof_summary.py $O/step $O/summary.md && sed -n '/Top kernels/,$p' $O/summary.md | head -30
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --kernel-include-regex 'gemm|Cijk|flash|attn' --output-format csv -d $O/pmc$i -o p -- python3 $R/bench.py --mode spmd --steps 2 --warmup 1 > $O/pmc_log$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $O/pmc_log$i.txt; exit 1; }
  echo "pass $i ok"
done
python3 $R/tools/gemm_pmc_table.py $O/pmc1 --md $O/pmc_mfma.md && python3 $R/tools/gemm_pmc_table.py $O/pmc2 --md $O/pmc_l2.md | head -5
