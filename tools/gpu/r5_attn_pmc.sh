#!/bin/bash
# PMC of the dK/dV kernel, production vs the MFMA+LDS-only ablation (ABL 7)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/attn_pmc5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for a in 0 7; do
CAAMD_FA64_BWD_ABL=$a timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVES --kernel-include-regex bwd_dkdv --output-format csv -d $O/a${a}p1 -- python3 $R/tools/bench_attn.py > $O/a${a}p1.log 2>&1 || { echo "p1 $a failed"; tail -5 $O/a${a}p1.log; exit 1; }
CAAMD_FA64_BWD_ABL=$a timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex bwd_dkdv --output-format csv -d $O/a${a}p2 -- python3 $R/tools/bench_attn.py > $O/a${a}p2.log 2>&1 || { echo "p2 $a failed"; tail -5 $O/a${a}p2.log; exit 1; }
done
find $O -name "*counter_collection.csv" | head
