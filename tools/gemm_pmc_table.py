"""Per-GEMM PMC table from rocprofv3 ``--pmc`` CSVs (one or more passes under a
directory): one row per (kernel, grid) over the profiled steps, with the
normalised MFMA utilisation

    util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x CUs x 4)

(GRBM_GUI_ACTIVE is summed over the 8 XCDs, MFMA busy counts cycles over all
SIMDs: MI355X_MICROARCH.md "s_memtime tick vs SQ PMC units", "DVFS give-back"),
the effective clock GUI/8/duration when the CSV carries timestamps, the L2 hit
rate and LDS bank-conflict share when those passes are present.

    python tools/gemm_pmc_table.py <dir> [--cus 256] [--md out.md]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0]
    for p in ("void ", "caamd::gemm::", "caamd::", "__amd_rocclr_"):
        n = n.replace(p, "")
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--md", default="")
    a = ap.parse_args()
    # (kernel, grid) -> counter -> [values]; durations per dispatch
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(dict)
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            key = (short(row.get("Kernel_Name", "?")), int(row.get("Grid_Size", 0) or 0) // max(1, int(row.get("Workgroup_Size", 1) or 1)))
            vals[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
            s, e = row.get("Start_Timestamp"), row.get("End_Timestamp")
            if s and e:
                durs[key][(f, row.get("Dispatch_Id"))] = (int(e) - int(s)) * 1e-9
    rows = []
    for key, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        d = list(durs[key].values())
        dur = sum(d) / len(d) if d else None
        gui = m.get("GRBM_GUI_ACTIVE")
        util = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui / 8 * a.cus * 4) if gui and "SQ_VALU_MFMA_BUSY_CYCLES" in m else None
        clk = gui / 8 / dur / 1e9 if gui and dur else None
        hit = (m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])) if "TCC_HIT_sum" in m else None
        bank = (m["SQ_LDS_BANK_CONFLICT"] / max(1.0, m["SQ_LDS_IDX_ACTIVE"])) if "SQ_LDS_BANK_CONFLICT" in m else None
        vpm = (m["SQ_INSTS_VALU"] / max(1.0, m["SQ_INSTS_MFMA"])) if "SQ_INSTS_MFMA" in m and "SQ_INSTS_VALU" in m else None
        rows.append((key, n, dur, util, clk, hit, bank, vpm))
    rows.sort(key=lambda r: -((r[2] or 0) * r[1]))
    f = lambda x, fmt: "-" if x is None else fmt.format(x)
    out = ["| kernel | WGs | dispatches | us (profiled) | MFMA util | clock GHz | L2 hit | LDS conflict/active | VALU/MFMA |",
           "|---|---|---|---|---|---|---|---|---|"]
    for (k, g), n, dur, util, clk, hit, bank, vpm in rows:
        out.append(f"| `{k}` | {g} | {n} | {f(dur and dur * 1e6, '{:.1f}')} | {f(util, '{:.3f}')} | "
                   f"{f(clk, '{:.2f}')} | {f(hit, '{:.3f}')} | {f(bank, '{:.3f}')} | {f(vpm, '{:.2f}')} |")
    text = "\n".join(out)
    print(text)
    if a.md:
        with open(a.md, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
