set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/attn_pmc
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/attn_pmc/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/attn_pmc/kt -- python3 $R/tools/attn_only.py > $R/gpurun_out/attn_pmc/kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/attn_pmc/p1 -- python3 $R/tools/attn_only.py > $R/gpurun_out/attn_pmc/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/attn_pmc/p2 -- python3 $R/tools/attn_only.py > $R/gpurun_out/attn_pmc/p2.log 2>&1
echo done $?
