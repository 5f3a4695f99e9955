#!/bin/bash
# PMC of the second-generation attention kernels (GPT-2-XL shape D=64, Llama prefill D=128)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/attn_pmc_r6
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CTR="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-include-regex fa64 --output-format csv -d $O/d64 -- python3 $R/tools/bench_attn.py > $O/d64.log 2>&1 || { echo "d64 failed"; tail -5 $O/d64.log; exit 1; }
python3 $R/tools/gemm_pmc_table.py $O/d64
