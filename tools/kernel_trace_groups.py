"""Group a rocprofv3 kernel-trace CSV by (kernel, grid, workgroup) and print count,
mean and total device time per group (largest total first): tells apart launches of
one kernel with different shapes (e.g. the decode GEMM's qkv / o / down grids).

    python tools/kernel_trace_groups.py run_kernel_trace.csv [--top 40]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    g = defaultdict(list)
    with open(path) as f:
        rd = csv.DictReader(f)
        cols = rd.fieldnames
        gx = next(c for c in cols if c.lower().startswith("grid_size_x") or c.lower() == "grid_size")
        wx = next((c for c in cols if c.lower().startswith("workgroup_size_x") or c.lower() == "workgroup_size"), None)
        for row in rd:
            name = row["Kernel_Name"][:90]
            key = (name, row[gx], row[wx] if wx else "")
            g[key].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1000.0)
    rows = sorted(g.items(), key=lambda kv: -sum(kv[1]))
    tot = sum(sum(v) for v in g.values())
    print(f"total kernel time {tot / 1000:.1f} ms")
    print(f"{'total_ms':>9} {'calls':>7} {'mean_us':>8} {'p50_us':>8}  grid  wg  kernel")
    for (name, grid, wg), v in rows[:top]:
        s = sorted(v)
        print(f"{sum(v) / 1000:9.2f} {len(v):7d} {sum(v) / len(v):8.2f} {s[len(s) // 2]:8.2f}  {grid} {wg}  {name}")


if __name__ == "__main__":
    main()
