#!/usr/bin/env python3
"""Per-wave timeline of one TB launch (s_memrealtime stamps, 100 MHz): how
long waves live relative to the launch, per XCD, per strip/chunk class.

    python tools/wave_timeline.py --nx 8192 --ny 8192 --depth 12
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parallel_heat_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=8192)
    ap.add_argument("--ny", type=int, default=8192)
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--variant", type=int, default=-1)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--interior", action="store_true", help="block inside a larger plate")
    ap.add_argument("--launches", type=int, default=4)
    ap.add_argument("--passes", type=int, default=40,
                    help="back-to-back launches timed with events: wall per pass vs one launch's span")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = ops.Geom(nx=a.nx, ny=a.ny) if not a.interior else \
        ops.Geom(nx=4 * a.nx, ny=4 * a.ny, gx0=a.nx, gy0=a.ny)
    x = ops.Field(a.nx, a.ny, a.depth, dev)
    y = ops.Field(a.nx, a.ny, a.depth, dev)
    ops.init_field(x, g, "random", 1)
    ops.init_field(y, g, "random", 1)
    cap = 1 << 16
    st = torch.full((cap * 4,), -1, dtype=torch.int64, device=dev)
    for _ in range(a.launches):  # warm
        ops.tb_step(x, y, g, a.depth, waves_target=a.waves, variant=a.variant)
        x, y = y, x
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.passes):
        ops.tb_step(x, y, g, a.depth, waves_target=a.waves, variant=a.variant)
        x, y = y, x
    e1.record()
    e1.synchronize()
    wall_us = e0.elapsed_time(e1) * 1e3 / max(1, a.passes)
    ops.tb_stamps(st)
    ops.tb_step(x, y, g, a.depth, waves_target=a.waves, variant=a.variant)
    torch.cuda.synchronize()
    ops.tb_stamps(None)
    s = st.view(-1, 4).cpu()
    s = s[s[:, 0] >= 0]
    t0 = int(s[:, 0].min())
    start = (s[:, 0] - t0).double() * 10e-3  # us
    end = (s[:, 1] - t0).double() * 10e-3
    dur = end - start
    blk = s[:, 2] >> 40
    xcc = (s[:, 2] >> 32) & 0xF
    hw = s[:, 2] & 0xFFFFFFFF
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    slot = ((xcc * 8 + se) * 16 + cu) * 4 + simd  # a SIMD of the chip
    # Pairs of waves sharing a SIMD: is the first-dispatched (older) one faster?
    order = torch.argsort(slot * 1_000_000 + blk)
    ss, bb, dd = slot[order], blk[order], dur[order]
    older, younger = [], []
    for i in range(len(ss) - 1):
        if ss[i] == ss[i + 1] and (i == 0 or ss[i - 1] != ss[i]):
            older.append(float(dd[i]))
            younger.append(float(dd[i + 1]))
    nb = int(blk.max()) + 1
    strip = s[:, 3] >> 32
    chunk = s[:, 3] & 0xFFFFFFFF
    span = float(end.max())
    nstr, nch = int(strip.max()) + 1, int(chunk.max()) + 1
    out = {
        "nx": a.nx, "ny": a.ny, "depth": a.depth, "waves": int(s.shape[0]), "span_us": round(span, 1),
        "wall_per_pass_us": round(wall_us, 1),
        "gap_us": round(wall_us - span, 1),
        "gcells_s_wall": round(a.nx * a.ny * a.depth / wall_us * 1e-3, 1),
        "mean_dur_us": round(float(dur.mean()), 1), "min_dur_us": round(float(dur.min()), 1),
        "max_dur_us": round(float(dur.max()), 1), "busy_fraction": round(float(dur.sum()) / (span * s.shape[0]), 3),
        "start_max_us": round(float(start.max()), 1),
        "end_p10_p50_p90_us": [round(float(end.quantile(q)), 1) for q in (0.1, 0.5, 0.9)],
        "xcd_last_end_us": [round(float(end[xcc == i].max()), 1) for i in range(8)],
        "xcd_mean_dur_us": [round(float(dur[xcc == i].mean()), 1) for i in range(8)],
        "edge_strip_mean_dur_us": round(float(dur[(strip == 0) | (strip == nstr - 1)].mean()), 1),
        "inner_strip_mean_dur_us": round(float(dur[(strip > 0) & (strip < nstr - 1)].mean()), 1),
        "edge_chunk_mean_dur_us": round(float(dur[(chunk == 0) | (chunk == nch - 1)].mean()), 1),
        "strips": nstr, "chunks": nch, "simds_used": int(slot.unique().numel()),
        "simd_pairs": len(older),
        "older_in_pair_mean_dur_us": round(sum(older) / max(1, len(older)), 1),
        "younger_in_pair_mean_dur_us": round(sum(younger) / max(1, len(younger)), 1),
        "first_half_blocks_mean_dur_us": round(float(dur[blk < nb // 2].mean()), 1),
        "second_half_blocks_mean_dur_us": round(float(dur[blk >= nb // 2].mean()), 1),
    }
    # Age rank of each wave on its SIMD (0 = first-dispatched block) and the
    # per-SIMD finish times: how the launch tail splits across ages.
    rank = torch.zeros_like(blk)
    prev, r = -1, 0
    for i in range(len(ss)):
        r = r + 1 if int(ss[i]) == prev else 0
        prev = int(ss[i])
        rank[order[i]] = r
    ages = []
    for a_ in range(int(rank.max()) + 1):
        m = rank == a_
        ages.append({"age": a_, "waves": int(m.sum()), "mean_start_us": round(float(start[m].mean()), 1),
                     "mean_dur_us": round(float(dur[m].mean()), 1),
                     "mean_end_us": round(float(end[m].mean()), 1)})
    out["by_age_rank"] = ages
    parts = []
    for q in range(4):  # grid quarters (the age groups of a 4-group launch)
        m = (blk >= q * nb // 4) & (blk < (q + 1) * nb // 4)
        parts.append({"quarter": q, "waves": int(m.sum()), "mean_dur_us": round(float(dur[m].mean()), 1),
                      "mean_rank": round(float(rank[m].double().mean()), 2)})
    out["by_grid_quarter"] = parts
    # The last waves to finish: what they are.
    idx = torch.argsort(end, descending=True)[:12]
    out["last_waves"] = [{"end_us": round(float(end[i]), 1), "dur_us": round(float(dur[i]), 1),
                          "strip": int(strip[i]), "chunk": int(chunk[i]), "rank": int(rank[i]),
                          "block": int(blk[i]), "xcc": int(xcc[i])} for i in idx.tolist()]
    hist = torch.histc(end.float(), bins=10, min=0, max=span)
    out["end_histogram_10"] = [int(x) for x in hist.tolist()]
    last = torch.zeros(int(slot.max()) + 1, dtype=torch.float64)
    last.index_reduce_(0, slot, end, "amax", include_self=False)
    used = last[torch.unique(slot)]
    out["simd_last_end_p10_p50_p90_us"] = [round(float(used.quantile(q)), 1) for q in (0.1, 0.5, 0.9)]
    # Row redundancy of the plan (classic plans: every chunk streams its rows
    # plus the K-1 rows of the trapezoid on each side, averaged over levels)
    # and the column redundancy of a 256-column strip with a K-column halo.
    ch = a.nx / nch
    out["row_redundancy"] = round((ch + a.depth - 1) / ch, 3)
    out["col_redundancy"] = round(a.ny and (256 * nstr) / a.ny, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
