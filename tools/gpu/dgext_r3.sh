#!/bin/bash
# Decode GEMM v3: in-kernel last-arriver split-K combine vs a separate reduce launch.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/dgext
mkdir -p $O
timeout -k 10 400 python -u tools/bench_decode_gemm3.py --ext --sweep > $O/bench.jsonl 2>&1; rc=$?
cat $O/bench.jsonl | grep -v '"check"' ; exit $rc
