#!/bin/bash
# skinny GEMM second generation: per-mode numerics (CAAMD_SKINNY_V=2/3/4) then a cache-cold sweep of the correct ones
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/skinny2
mkdir -p $O
for v in 1 2 3 4; do
  CAAMD_SKINNY_V=$v timeout -k 10 120 python -u - > $O/num_v$v.log 2>&1 <<'PY' || { tail -20 $O/num_v$v.log; exit 1; }
import os, torch
from cluster_anywhere_amd.ops.llm import skinny_linear, skinny_splits
out = []
for M in (1, 32, 128):
    for N, K in ((6144, 4096), (4096, 14336), (28672, 4096)):
        torch.manual_seed(M + N)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
        ref = x.float() @ w.float().t()
        y = skinny_linear(x, w).float()
        err = ((y - ref).norm() / ref.norm()).item()
        bad = ((y - ref).abs() > 0.05 * ref.abs().max()).nonzero()
        out.append(f"M{M} N{N} K{K} s{skinny_splits(N, K)} err={err:.4f} bad_rows={sorted(set(bad[:, 0].tolist()))[:6]} bad_cols_mod64={sorted(set((bad[:, 1] % 64).tolist()))[:8]} n={len(bad)}")
print(f"v={os.environ['CAAMD_SKINNY_V']}"); print("\n".join(out))
PY
  cat $O/num_v$v.log | grep -v amdgpu.ids
done
for v in 1 2 3 4; do
  CAAMD_SKINNY_V=$v timeout -k 10 200 python -u tools/bench_decode_gemm.py > $O/dgemm_v$v.log 2>&1 || { tail -20 $O/dgemm_v$v.log; exit 1; }
  echo "v=$v"; grep gemm $O/dgemm_v$v.log | python3 -c "import sys,json; [print(d['gemm'], d['splits'], d['hipblaslt_us'], d['ours_us'], d['ours_TBps'], d['rel_err']) for d in map(json.loads, sys.stdin)]"
done
