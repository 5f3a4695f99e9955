#!/bin/bash
# Round 4: compile-time mask split in the D=64 attention kernels -- tests, then old/new .so alternating.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/attn_ab
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 120 python -u tools/bench_attn.py > $O/new_$i.json 2>&1 || { echo "new failed"; tail -5 $O/new_$i.json; exit 1; }
  echo "new: $(tail -1 $O/new_$i.json)"
  ATTN_SO=tools/gpu/fa_old/_C_old.so timeout -k 10 120 python -u tools/bench_attn.py > $O/old_$i.json 2>&1 || { echo "old failed"; tail -5 $O/old_$i.json; exit 1; }
  echo "old: $(tail -1 $O/old_$i.json)"
done
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail -10 $O/bench_$i.log; exit 1; }
  echo "step: $(grep -o '"value": [0-9.]*' $O/bench_$i.log)"
done
