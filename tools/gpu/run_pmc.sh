cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 --list-avail > gpurun_out/pmc/avail.txt 2>&1 || true
cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $GRAFT_REPO_ROOT/gpurun_out/pmc/g$i -o run -- python $GRAFT_REPO_ROOT/tools/attn_only.py > $GRAFT_REPO_ROOT/gpurun_out/pmc/g$i.log 2>&1 || echo "group $i failed"
done
echo done
