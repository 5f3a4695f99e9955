#!/bin/bash
# Counter passes over one GEMM shape (args: layout M N K bm bn algo tag). Each pass
# its own rocprofv3 run (gpurun rule: counters per block within limits).
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=$1; M=$2; N=$3; K=$4; BM=$5; BN=$6; A=$7; TAG=$8
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_MFMA"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex gemm --output-format csv -d $OUT -o p$i -- python3 tools/gemm_one.py $L $M $N $K $BM $BN $A > $OUT/log$i.txt 2>&1
done
python3 tools/prof_summarize.py $OUT
