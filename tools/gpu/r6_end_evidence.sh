#!/bin/bash
# Round 6 end: per-GEMM PMC pass (MFMA util) on the final tree + RLlib bench refresh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/end_evidence
mkdir -p $O
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 240 rocprofv3 --pmc $P1 --kernel-trace --kernel-include-regex 'gemm|flash|attn|fa64' --output-format csv -d $O/pmc1 -o p -- python3 $R/bench.py --mode spmd --steps 2 --warmup 1 > $O/pmc_log1.txt 2>&1 || { echo "pmc pass failed"; tail -5 $O/pmc_log1.txt; exit 1; }
python3 $R/tools/gemm_pmc_table.py $O/pmc1 --md $O/pmc_mfma.md | head -30
cd $R
timeout -k 10 300 python -u tools/bench_rllib.py --runners 4 --envs-per-runner 96 --runner-gpus 0.1 --seconds 25 > $O/rllib.log 2>&1 || { tail -20 $O/rllib.log; exit 1; }
grep -E '^\{' $O/rllib.log | tail -1
