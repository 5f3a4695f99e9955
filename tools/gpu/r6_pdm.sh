#!/bin/bash
# Round 6: paged decode at four blocks per CU (CAAMD_PDM_OCC4) -- tests, serving A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_pdm
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py tests/test_llama_hf_parity_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
for i in 1 2; do for f in 1 0; do
  CAAMD_PDM_OCC4=$f timeout -k 10 240 python3 -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/b_${f}_$i.log 2>&1 || { tail -20 $O/b_${f}_$i.log; exit 1; }
  echo "pdm_occ4=$f $(grep -o '"value": [0-9.]*\|"steady_tpot_p50_ms": [0-9.]*\|"ttft_p50_s": [0-9.]*' $O/b_${f}_$i.log | tr '\n' ' ')"
done; done
