#!/bin/bash
# kernel-trace of the serving bench (one-step-ahead decode)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/llmp -o run -- python3 -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > gpurun_out/llmp.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/llmp.log; exit 1; }
grep metric gpurun_out/llmp.log | cut -c1-300
mkdir -p gpurun_out/llmp && cp $(find /tmp/llmp -name "*kernel_stats.csv") gpurun_out/llmp/
