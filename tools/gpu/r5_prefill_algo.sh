#!/bin/bash
# prefill GEMM algo sweep at the 8192-token chunk the serving bench uses
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/bench_prefill_gemm.py --tokens 8192 --algos 9,4009,1009,3009 > gpurun_out/prefill_algo_8192.jsonl 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/prefill_algo_8192.jsonl; exit 1; }
grep '"gemm"' gpurun_out/prefill_algo_8192.jsonl
