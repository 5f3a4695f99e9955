#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6_algo
timeout -k 10 300 python -u tools/gemm_algo_ab.py > gpurun_out/r6_algo/ab.jsonl 2>&1 || { tail -5 gpurun_out/r6_algo/ab.jsonl; exit 1; }
grep shape gpurun_out/r6_algo/ab.jsonl
