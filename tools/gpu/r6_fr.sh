#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/fr
timeout -k 10 120 python -u tools/probe_fused_random.py > gpurun_out/fr/fr.jsonl 2> gpurun_out/fr/err.log || { tail -5 gpurun_out/fr/err.log; exit 1; }
cat gpurun_out/fr/fr.jsonl
