"""Summarise a rocprofv3 ``--kernel-trace --stats`` CSV directory into markdown
(top kernels by total time, grouped into families), for profiles/."""
import csv
import glob
import os
import sys


def family(name: str) -> str:
    n = name
    if n.startswith("Cijk_") or n.startswith("Custom_Cijk"):
        return "GEMM (hipBLASLt)"
    for key, fam in [("gemm_pp_kernel", "GEMM MFMA (ours)"), ("gemm_sk_kernel", "GEMM MFMA wgrad (ours)"), ("gemm_kernel", "GEMM MFMA (ours)"),
                     ("transpose_bf16", "weight transpose (ours)"), ("fa_fwd", "flash-attn fwd (ours)"), ("fa_bwd_dq", "flash-attn dQ (ours)"),
                     ("fa_bwd_dkdv", "flash-attn dK/dV (ours)"), ("fa6410fwd_kernel", "flash-attn fwd (ours)"),
                     ("fa64::fwd_kernel", "flash-attn fwd (ours)"), ("bwd_dq_kernel", "flash-attn dQ (ours)"),
                     ("bwd_dkdv_kernel", "flash-attn dK/dV (ours)"), ("rowsum_partial", "column reduce (ours)"), ("ln_fwd", "LayerNorm fwd (ours)"),
                     ("ln_bwd", "LayerNorm bwd (ours)"), ("colsum", "column reduce (ours)"),
                     ("bias_gelu", "bias+GELU (ours)"), ("xent", "cross-entropy (ours)"),
                     ("adamw", "fused AdamW (ours)"), ("sumsq", "grad-norm (ours)"),
                     ("conv_kernel", "conv MFMA (ours)"), ("maxpool3s2", "vision (ours)"),
                     ("normalize_pad8", "vision (ours)"), ("igemm_fwd", "conv (MIOpen)"), ("bias_act", "bias/act (ours)"),
                     ("nccl", "RCCL"), ("rccl", "RCCL"), ("reduce_kernel", "torch reduce"),
                     ("elementwise", "torch elementwise"), ("Cat", "torch cat"),
                     ("copyBuffer", "memcpy"), ("fillBuffer", "memset")]:
        if key in n:
            return fam
    return "other"


def main(d, out):
    fs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if fs:
        rows = list(csv.DictReader(open(fs[0])))
    else:  # rocprofv3 7.x default output: rocpd SQLite database
        import sqlite3

        db = sqlite3.connect(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0])
        q = ("select name, count(*), sum(duration) from kernels group by name "
             "order by sum(duration) desc")
        rows = [{"Name": n, "Calls": c, "TotalDurationNs": t, "AverageNs": t / c, "Percentage": 0.0}
                for n, c, t in db.execute(q)]
        tot_ = sum(r["TotalDurationNs"] for r in rows)
        for r in rows:
            r["Percentage"] = 100.0 * r["TotalDurationNs"] / tot_
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    fam = {}
    for r in rows:
        k = family(r["Name"])
        fam[k] = fam.get(k, 0.0) + float(r["TotalDurationNs"])
    lines = [f"# rocprofv3 kernel summary ({os.path.basename(d)})", "",
             f"Total GPU kernel time: {tot / 1e6:.2f} ms", "", "## By family", "",
             "| family | ms | % |", "|---|---|---|"]
    for k, v in sorted(fam.items(), key=lambda x: -x[1]):
        lines.append(f"| {k} | {v / 1e6:.2f} | {100 * v / tot:.1f} |")
    lines += ["", "## Top kernels", "", "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in rows[:25]:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:20]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
