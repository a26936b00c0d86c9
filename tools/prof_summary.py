#!/usr/bin/env python3
"""Summarise rocprofv3 output (kernel-trace CSV/DB and PMC CSVs) into a
markdown file under profiles/.

    python tools/prof_summary.py --trace gpurun_out/prof --pmc gpurun_out/pmc --out profiles/x.md
"""
import argparse
import collections
import csv
import glob
import os
import sqlite3


def kernel_stats(trace_dir):
    rows = []
    for f in glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                         r.get("VGPR_Count", ""), r.get("Grid_Size", r.get("Grid_Size_X", ""))))
    for f in glob.glob(os.path.join(trace_dir, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        for name, dur in c.execute("select name, duration from kernels"):
            rows.append((name, int(dur), "", ""))
    agg = collections.defaultdict(list)
    for name, dur, vg, grid in rows:
        agg[name].append(dur)
    total = sum(sum(v) for v in agg.values()) or 1
    out = []
    for name, durs in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        out.append((name, len(durs), sum(durs) / len(durs) / 1e3, sum(durs) / 1e3, 100 * sum(durs) / total))
    return out


def pmc(pmc_dir, match):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if match in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", default=None)
    ap.add_argument("--pmc", default=None)
    ap.add_argument("--match", default="tb_kernel")
    ap.add_argument("--title", default="rocprofv3 summary")
    ap.add_argument("--note", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    lines = [f"# {a.title}", ""]
    if a.note:
        lines += [a.note, ""]
    if a.trace:
        lines += ["## Kernel trace (per-kernel time)", "",
                  "| kernel | calls | avg us | total us | % |", "|---|---|---|---|---|"]
        for name, n, avg, tot, pct in kernel_stats(a.trace):
            lines.append(f"| `{name[:110]}` | {n} | {avg:.1f} | {tot:.1f} | {pct:.1f} |")
        lines.append("")
    if a.pmc:
        c = pmc(a.pmc, a.match)
        lines += [f"## Hardware counters (mean per dispatch of `{a.match}`)", "",
                  "| counter | value |", "|---|---|"]
        for k in sorted(c):
            lines.append(f"| {k} | {c[k]:.4g} |")
        if "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            lines += ["", "Derived (fractions of wave lifetime, SQ quad-cycle counters):", ""]
            for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if k in c:
                    lines.append(f"* {k} / SQ_WAVE_CYCLES = {c[k] / wc:.2f}")
        if "FETCH_SIZE" in c:
            lines.append(f"* HBM read bytes (2 x FETCH_SIZE, gfx950 calibration) = {2 * c['FETCH_SIZE'] * 1024 / 1e6:.1f} MB per dispatch")
        if "WRITE_SIZE" in c:
            lines.append(f"* HBM write bytes (WRITE_SIZE) = {c['WRITE_SIZE'] * 1024 / 1e6:.1f} MB per dispatch")
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            h, m = c["TCC_HIT_sum"], c["TCC_MISS_sum"]
            lines.append(f"* L2 hit rate = {h / (h + m):.2f}")
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    open(a.out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
