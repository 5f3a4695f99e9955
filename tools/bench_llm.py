"""Offline LLM serving throughput on one MI355X (BASELINE.json config
"Ray Serve Llama-3-8B bf16, one replica per MI355X, continuous batching"):
random-init Llama-3-8B, synthetic prompts, continuous batching engine.

python tools/bench_llm.py --model llama3-8b --num-prompts 256 --input-len 512 --output-len 256
Prints one JSON line: output tokens/s, total tokens/s, TTFT/TPOT percentiles.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cluster_anywhere_amd.llm import LLMEngine, SamplingParams  # noqa: E402
from cluster_anywhere_amd.models.llama import Llama, LlamaConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--num-prompts", type=int, default=256)
    ap.add_argument("--input-len", type=int, default=512)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    # prefill chunk (tokens per prefill step): 8192 -> TTFT p50 1.774 vs 1.870 s at 16384,
    # output tok/s 9786 vs 9807 (profiles/llm_prefill_chunk_r5.jsonl)
    ap.add_argument("--max-batched-tokens", type=int, default=8192)
    ap.add_argument("--no-graphs", action="store_true")
    a = ap.parse_args()
    cfg = LlamaConfig.named(a.model)
    torch.manual_seed(0)
    with torch.device("cuda"):
        m = Llama(cfg).to(torch.bfloat16)
    m.init_weights(std=0.02)
    eng = LLMEngine(m, max_num_seqs=a.max_num_seqs, max_model_len=a.input_len + a.output_len + 16,
                    max_num_batched_tokens=a.max_batched_tokens, use_graphs=not a.no_graphs)
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(0, cfg.vocab_size, (a.input_len,), generator=g).tolist() for _ in range(a.num_prompts)]
    sp = SamplingParams(max_tokens=a.output_len, ignore_eos=True)
    # warmup: captures graphs for the buckets used later
    eng.generate(prompts[: min(8, len(prompts))], SamplingParams(max_tokens=8, ignore_eos=True))
    for b in (1, 2, 4, 8, 16, 32, 64, 128, 256):
        if b <= a.max_num_seqs and eng.use_graphs:
            eng._graph_for(b)
    torch.cuda.synchronize()
    eng.decode_times.clear()
    t0 = time.time()
    outs = eng.generate(prompts, sp)
    torch.cuda.synchronize()
    dt = time.time() - t0
    n_out = sum(len(o.output_token_ids) for o in outs)
    n_in = sum(len(o.prompt_token_ids) for o in outs)
    ttft = sorted(o.metrics["first_token"] - o.metrics["arrival"] for o in outs)
    tpot = sorted((o.metrics["now"] - o.metrics["first_token"]) / max(1, len(o.output_token_ids) - 1) for o in outs)
    print(json.dumps({
        "metric": "Serve LLM offline throughput (Llama-3-8B, continuous batching)", "model": a.model,
        "value": round(n_out / dt, 1), "unit": "output tokens/s", "total_tokens_per_s": round((n_in + n_out) / dt, 1),
        "num_prompts": a.num_prompts, "input_len": a.input_len, "output_len": a.output_len,
        "elapsed_s": round(dt, 2), "ttft_p50_s": round(ttft[len(ttft) // 2], 3),
        "tpot_p50_ms": round(1000 * tpot[len(tpot) // 2], 2), "kv_blocks": eng.num_blocks,
        "preemptions": eng.stats["preemptions"], "graphs": eng.use_graphs, "dtype": "bf16",
        "max_num_seqs": a.max_num_seqs, **_steady(eng.decode_times, a.max_num_seqs),
        "data": "synthetic prompts, random-init weights"}))


def _steady(times, max_seqs):
    """Steady-state decode: steps that ran with (nearly) the full batch; the step
    latency there is the time between two tokens of every running sequence."""
    full = sorted(t for b, t in times if b >= 0.9 * max_seqs)
    if not full:
        return {"steady_decode_steps": 0}
    return {"steady_decode_steps": len(full), "steady_batch": max_seqs,
            "steady_tpot_p50_ms": round(1000 * full[len(full) // 2], 2),
            "steady_tpot_p90_ms": round(1000 * full[int(len(full) * 0.9)], 2),
            "steady_decode_tokens_per_s": round(max_seqs / full[len(full) // 2], 1)}


if __name__ == "__main__":
    main()
