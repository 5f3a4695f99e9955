#!/bin/bash
# decode GEMM bound probe: slab count, batch rows and ring depths (tools/dg_probe.py)
set -o pipefail
mkdir -p gpurun_out/dgprobe
for r in 0 1 2; do
  CAAMD_DG_RING=$r timeout -k 10 240 python -u tools/dg_probe.py >> gpurun_out/dgprobe/probe.jsonl 2>> gpurun_out/dgprobe/err.log || exit $?
done
cat gpurun_out/dgprobe/probe.jsonl
