#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/transpose
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/transpose/tests.log 2>&1; rc=$?
tail -2 gpurun_out/transpose/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/bench_transpose.py > gpurun_out/transpose/t.jsonl 2>&1 || { tail -5 gpurun_out/transpose/t.jsonl; exit 1; }
cat gpurun_out/transpose/t.jsonl
