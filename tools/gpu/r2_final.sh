#!/bin/bash
# end-of-round checks: full GPU suite, smoke, headline bench, cache-cold decode GEMM sweep
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log
for s in 0 1 2 4 8; do
  CAAMD_SKINNY_SPLITS=$s timeout -k 10 200 python -u tools/bench_decode_gemm.py > $O/dgemm_s$s.log 2>&1 || { tail -20 $O/dgemm_s$s.log; exit 1; }
  echo "splits=$s"; grep gemm $O/dgemm_s$s.log | cut -c1-220
done
