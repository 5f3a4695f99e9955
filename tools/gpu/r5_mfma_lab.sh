#!/bin/bash
# MFMA dependency / block-structure microbenchmark + dK/dV kernel time (production vs fully stripped)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/lab/mfma_dep_bench > gpurun_out/mfma_dep2.txt 2>&1 || { echo "lab failed"; cat gpurun_out/mfma_dep2.txt; exit 1; }
cat gpurun_out/mfma_dep2.txt
for a in 0 31; do
CAAMD_FA64_BWD_ABL=$a timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/abl$a -o run -- python3 -u tools/bench_attn.py > gpurun_out/abl$a.log 2>&1 || { echo "abl $a failed"; tail -20 gpurun_out/abl$a.log; exit 1; }
grep bwd_us gpurun_out/abl$a.log
f=$(find gpurun_out/abl$a -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if "fa64" in n or "flash" in n:
        print(n[:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg")
PY
done
