"""Per-kernel time inside a time window of a rocprofv3 kernel trace (e.g. the
steady decode phase of an LLM run, after the prefill burst).

    python tools/prof_window.py <rocprof dir> [--from-frac 0.5] [--to-frac 1.0] [--top 30]

Prints total / count / mean per kernel over dispatches that START inside the
window (fractions of the traced span), plus the busy fraction of the window.
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--from-frac", type=float, default=0.5)
    ap.add_argument("--to-frac", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    if not rows:
        print("no kernel trace found")
        return
    rows.sort()
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    lo = t0 + a.from_frac * (t1 - t0)
    hi = t0 + a.to_frac * (t1 - t0)
    agg = defaultdict(lambda: [0, 0])
    busy = 0
    for s, e, n in rows:
        if lo <= s < hi:
            agg[n][0] += e - s
            agg[n][1] += 1
            busy += e - s
    span = hi - lo
    print(f"window {(hi - lo) / 1e6:.1f} ms, kernel busy {busy / 1e6:.1f} ms ({100 * busy / span:.1f} %)")
    print(f"{'total ms':>10} {'calls':>7} {'mean us':>9}  kernel")
    for n, (tot, cnt) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{tot / 1e6:10.2f} {cnt:7d} {tot / cnt / 1e3:9.1f}  {n[:110]}")


if __name__ == "__main__":
    main()
