#!/bin/bash
# Round 6 call E: library kernel names / times of the tuned plain NT GEMMs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_e
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r6e -o run -- python3 $R/tools/lib_gemm_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
f=$(find /tmp/r6e -name "*kernel_stats.csv" | head -1)
cp $f $O/kernel_stats.csv
cut -d, -f1-6 $O/kernel_stats.csv | head -20
