#!/bin/bash
# (historical: the A/B environment knob this script sets was removed after the measurement;
#  the script records how the committed profile was produced)
# Round 4: wave priority (s_setprio) placement in the dK/dV kernel: none / MFMA bursts / VALU pass.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/attn_prio
mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in 1 2; do
  CAAMD_FA64_PRIO=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or attn" > $O/pytest$v.log 2>&1; rc=$?
  tail -1 $O/pytest$v.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest$v.log | head -20; exit $rc; }
done
for i in 1 2; do
  for v in 0 1 2; do
    CAAMD_FA64_PRIO=$v timeout -k 10 120 python -u tools/bench_attn.py > $O/k${v}_$i.json 2>&1 || { echo "attn $v failed"; tail -5 $O/k${v}_$i.json; exit 1; }
    echo "prio=$v: $(tail -1 $O/k${v}_$i.json)"
  done
done
