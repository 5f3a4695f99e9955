#!/bin/bash
# kernel times of the decode path with the fused reduce + residual + RMSNorm launch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for f in 1 0; do
CAAMD_DECODE_REDUCE_NORM=$f timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rnp$f -o run -- python3 -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > gpurun_out/rnp$f.log 2>&1 || { echo "prof $f failed"; tail -20 gpurun_out/rnp$f.log; exit 1; }
grep metric gpurun_out/rnp$f.log | cut -c1-300
mkdir -p gpurun_out/rnp$f && cp $(find /tmp/rnp$f -name "*kernel_stats.csv") gpurun_out/rnp$f/
done
