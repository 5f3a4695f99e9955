#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/epiocc
timeout -k 10 240 python -u tools/gemm_epi_occupancy.py > gpurun_out/epiocc/occ.jsonl 2> gpurun_out/epiocc/err.log || { tail -5 gpurun_out/epiocc/err.log; exit 1; }
cat gpurun_out/epiocc/occ.jsonl
