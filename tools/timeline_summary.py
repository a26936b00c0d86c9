#!/usr/bin/env python3
"""Per-rank device timeline of a multi-rank run from rocprofv3 kernel traces.

    python tools/timeline_summary.py gpurun_out/r5g/tl --out profiles/r5_timeline_8ranks.md

Input: one rocprofv3 output per rank (`--kernel-trace --marker-trace
--output-format csv -o rank_%pid%`, each rank of the torchrun job under its own
rocprofv3; tools/sessions/sessions_r5g.sh).  Ranks are told apart by their process ids
and numbered in pid order.  Each kernel is classed as

  exchange  RCCL kernels (ncclDevKernel*, the grouped send/recv and the
            all-reduce) and the halo pack / unpack / box-copy launches,
  compute   the stencil kernels (TB streaming, level-split, tile, resident),
  other     init, checksum, judge, copies.

For the last complete timed bench step of every rank (the kernels between the
rank's last two "heat.run" roctx ranges when present, else its last 1000-step
window of stencil kernels) it prints the ordered phases with start/end in us
relative to the step's first kernel, the per-rank sums, and a coarse ASCII
gantt (one row per rank, E = exchange, C = compute, . = idle), the analogue
of the reference's Paraver timelines (Heat.pdf pp.8-11).
"""
import argparse
import collections
import csv
import glob
import os
import re
import sys


def classify(name):
    n = name.lower()
    if "nccl" in n or "pack" in n or "box_copy" in n or "copy_boxes" in n:
        return "exchange"
    if any(k in n for k in ("tb_kernel", "tb_split_kernel", "tile_kernel", "tile_resident",
                            "lds_kernel", "naive_kernel", "mfma")):
        return "compute"
    return "other"


def load(dirpath):
    ranks = collections.defaultdict(lambda: {"kernels": [], "markers": []})
    for f in glob.glob(os.path.join(dirpath, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            pid = int(r.get("Process_Id") or r.get("Pid") or re.findall(r"(\d+)", os.path.basename(f))[-1])
            ranks[pid]["kernels"].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                          r["Kernel_Name"]))
    for f in glob.glob(os.path.join(dirpath, "**", "*marker_api_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            pid = int(r.get("Process_Id") or r.get("Pid") or re.findall(r"(\d+)", os.path.basename(f))[-1])
            name = r.get("Function") or r.get("Operation") or r.get("Name") or ""
            ranks[pid]["markers"].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    return ranks


def window(rank):
    ks = sorted(rank["kernels"])
    runs = sorted((a, b) for a, b, n in rank["markers"] if n == "heat.run")
    if len(runs) >= 2:
        a0 = runs[-1][0]
        sel = [k for k in ks if k[0] >= a0]
        if sel:
            return sel
    comp = [k for k in ks if classify(k[2]) == "compute"]
    return [k for k in ks if comp and k[0] >= comp[max(0, len(comp) - 100)][0]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    ap.add_argument("--width", type=int, default=100)
    a = ap.parse_args()
    ranks = load(a.dir)
    if not ranks:
        print("no kernel traces under", a.dir, file=sys.stderr)
        return 1
    lines = ["# Per-rank device timeline (rocprofv3 kernel trace, one rocprofv3 per rank)", ""]
    wins = {}
    for i, pid in enumerate(sorted(ranks)):
        wins[i] = (pid, window(ranks[pid]))
    t0 = min(w[0][0] for _, w in wins.values() if w)
    t1 = max(w[-1][1] for _, w in wins.values() if w)
    span = max(1, t1 - t0)
    lines += [f"Window: the last timed step of each rank; {len(wins)} ranks; "
              f"{span / 1e3:.1f} us from the first rank's first kernel to the last rank's last.", "",
              "| rank (pid) | kernels | exchange us | compute us | other us | busy / window |",
              "|---|---|---|---|---|---|"]
    gantt = []
    for i, (pid, w) in wins.items():
        tot = collections.Counter()
        for s, e, n in w:
            tot[classify(n)] += e - s
        wspan = (w[-1][1] - w[0][0]) if w else 1
        busy = sum(tot.values())
        lines.append(f"| {i} ({pid}) | {len(w)} | {tot['exchange'] / 1e3:.1f} | "
                     f"{tot['compute'] / 1e3:.1f} | {tot['other'] / 1e3:.1f} | "
                     f"{busy / max(1, wspan):.2f} |")
        row = ["."] * a.width
        for s, e, n in w:
            c = {"exchange": "E", "compute": "C"}.get(classify(n), "o")
            lo = int((s - t0) * a.width / span)
            hi = max(lo + 1, int((e - t0) * a.width / span))
            for x in range(max(0, lo), min(a.width, hi)):
                if row[x] == "." or c == "E":
                    row[x] = c
        gantt.append(f"rank {i} |{''.join(row)}|")
    lines += ["", "```", *gantt, "```", "",
              "Phase sequence of rank 0 (us from its window start):", "", "| # | phase | start | end | kernel |",
              "|---|---|---|---|---|"]
    pid0, w0 = wins[0]
    base = w0[0][0] if w0 else 0
    for j, (s, e, n) in enumerate(w0[:60]):
        lines.append(f"| {j} | {classify(n)} | {(s - base) / 1e3:.1f} | {(e - base) / 1e3:.1f} | "
                     f"{n[:70]} |")
    text = "\n".join(lines) + "\n"
    if a.out:
        open(a.out, "w").write(text)
    print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
