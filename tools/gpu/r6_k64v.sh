#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6_k64v
timeout -k 10 400 python -u tools/gemm_k64_variants.py > gpurun_out/r6_k64v/ab.jsonl 2>&1 || { tail -5 gpurun_out/r6_k64v/ab.jsonl; exit 1; }
grep shape gpurun_out/r6_k64v/ab.jsonl
