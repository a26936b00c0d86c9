"""Strong-scaling model of a decomposed run on one MI355X node.

The reference quantifies its MPI scaling by hand (Heat.pdf p.5 Table 1:
speedup and efficiency at 1 and 10 machines; p.8-11 Paraver phases).  Here
the same accounting is a model that ``bench.py`` prints next to the measured
multi-GPU number, and that the autotune uses to skip candidates it rules out:

    time per 1000 iterations = compute(per-rank block) + exchanges x t_exchange
                               + checks x t_allreduce

* compute: the per-rank block's cells (plus the deep-halo ghost rows it
  recomputes) at the rate one MI355X reaches on a plate of that shape.  The
  rates are this build's measured whole-solver ``bench.py`` plates whose top
  and bottom rows are plate edges (the slowest rank of a decomposition,
  which the max over ranks reports), interpolated in strip-rows per SIMD --
  the planner's own measure of the work per launch (RESIDENT_POINTS when
  the span's box has a one-round resident plan, STREAM_POINTS otherwise).
* exchange: one grouped RCCL send/recv phase per m*K steps (deep halos),
  every message on its own xGMI link (full mesh, one hop): a fixed latency
  plus the largest message over the link bandwidth (XGMI).  2-D grids add
  the pack / unpack launches of the E/W columns and ghost corners.
* all-reduce: one 4-byte ncclAllReduce(max) per convergence check.

All parameters are stated in ``XGMI`` / ``*_POINTS`` and returned with
every prediction, so a measured SCALE record can be read against them.
``fit_exchange`` replaces XGMI's latency and bandwidth with values fitted to
grouped exchanges timed on the real ranks (bench.py does this before it
prunes autotune candidates; the measured points are in the JSON line).
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

from ..models.config import HeatConfig
from .topology import dims_create

# Exchange cost model on the xGMI full mesh (7 links x ~153 GB/s per GPU,
# SURVEY §2.4).  Latency: a grouped ncclSend/ncclRecv phase captured in a
# graph is O(10 us) of launch + protocol; bandwidth: the effective one-way
# rate RCCL's P2P transport reaches on one link at 0.1-1 MB messages.
XGMI = {
    "latency_us": 12.0,          # per grouped exchange phase
    "link_gbps": 50.0,           # effective GB/s per link and direction
    "pack_us": 3.0,              # per pack or unpack launch (2-D grids: 2 per exchange)
    "allreduce_us": 12.0,        # one 4-byte ncclAllReduce(max) per check
}

# Whole-solver rate (Tcells/s) of one MI355X on a bench plate (plate edges
# top and bottom) vs strip-rows per SIMD of that plate (232 useful columns
# per 256-column strip at depth 12, 1024 SIMDs), in two families: spans whose
# box has a one-dispatch-round resident plan (every tile co-resident for all
# passes between exchanges, tb_resident.hip) and the rest (level-split
# pipelines / per-pass tiles).  Resident points are long-span rates of the
# span BOX (multi-rank spans pay SPAN_COST below); the rest are rates of the
# owned block.  Enqueued bench steps, rounds 5-6 (profiles/r5_raw/r5h_*.txt,
# r5f_b*.txt, profiles/r6_raw/r6d/, r6f/, r6o/ - r6q/).
RESIDENT_POINTS: List[tuple] = [
    (18.0, 3.0),    # 512 x 8192 (16-GPU-like blocks; extrapolated, unmeasured)
    (36.0, 4.40),   # 1024 x 8192 4.33-4.45 / 2048 x 4096 4.42-4.47 (12 x 16 tiles, DPP, edge modes, r6o-q)
    (38.5, 4.90),   # 2192 x 4168 (the 4 x 2 8-GPU box at m = 7): 4.40-4.51 at 7-pass spans
    (41.0, 5.14),   # 1168 x 8192 (the 8 x 1 8-GPU box at m = 7, 7 full chunks): 4.67 at 7
    (72.0, 5.30),   # 2048 x 8192 5.25-5.34 / 4096^2 5.22-5.34 / 4144^2 5.37 (20 x 16)
]
STREAM_POINTS: List[tuple] = [
    (18.0, 3.0),    # extrapolated, unmeasured
    (36.0, 3.3),    # 1024 x 8192 per-pass tiles (round 3/4: 3.23)
    (72.0, 3.90),   # 2048 x 8192 3.90 / 4096 x 4096 3.90, split pipelines
    (144.0, 4.85),  # 4096 x 8192 4.76-4.91 (2 GPUs, plain rows)
    (288.0, 5.15),  # 8192 x 8192 5.13-5.25 (1 GPU, streaming rows, profiles/r5_stores.md)
]
RATE_POINTS = STREAM_POINTS  # the large-block end (1 GPU) is a stream plate

# A resident span of m passes pays one whole-tile load and store (what a
# per-pass tile launch pays every pass): a rank's resident rate at m passes
# per exchange is the long-span plate rate above / (1 + SPAN_COST / m).
# Round-6 plates with the span capped (HEAT_TB_RES_SPAN, profiles/r6_raw/r6d):
# 4144^2 (20 x 16 tiles) 5.37 long, 4.84 / 4.78 / 4.54 / 4.22 at 5 / 4 / 3 /
# 2 passes (fit: 0.55); 1192 x 8192 (14 x 8) 4.29 long, 3.90 at 8 (0.8).
SPAN_COST = 0.7

SIMDS = 1024
STRIP_COLS = 232  # useful columns per 256-column strip at depth 12
CUS = 256

# The resident planner's shapes (rows per wave, waves, workgroups per CU at
# their VGPR budget): csrc/kernels/tb_resident.hip plan_res.
RES_SHAPES = [(12, 8, 2), (13, 8, 2), (14, 8, 2), (16, 8, 2), (20, 8, 1), (24, 8, 1),
              (12, 16, 1), (20, 16, 1)]


def _tile_step_estimate(units: int, occ: int, rows: int, waves: int) -> float:
    """csrc/kernels/tb_tile.hpp tile_step_estimate (the planner's choice)."""
    cap = CUS * occ
    full = (units - 1) // cap
    busiest = (units - full * cap + CUS - 1) // CUS

    def cost(tiles):
        wps = tiles * waves / 4.0
        return wps * rows * (2.7 if wps >= 4.0 else 3.1)
    return full * cost(occ) + cost(busiest)


def resident_shape(rows: int, cols: int, depth: int = 12) -> tuple:
    """The resident planner's (rows per wave, waves) for a rows x cols box, or
    None without a one-round plan (csrc/src/topology.cpp
    resident_shape_static, tb_resident.hip plan_res)."""
    if rows <= 0 or cols <= 0 or depth < 4 or depth % 2:
        return None
    strips = math.ceil(cols / (256 - 2 * ((depth + 3) // 4 * 4)))
    best, best_est, best_h = None, 0.0, 0
    for r, nw, occ in RES_SHAPES:
        h = r * nw - 2 * depth
        if h < max(depth, 4):
            continue
        units = strips * math.ceil(rows / h)
        if units > CUS * occ:
            continue
        est = _tile_step_estimate(units, occ, r, nw)
        if best is None or est < best_est:
            best, best_est, best_h = (r, nw), est, h
    if best is not None and math.ceil(rows / math.ceil(rows / best_h)) < depth:
        return None
    return best


def resident_fits(rows: int, cols: int, depth: int = 12) -> bool:
    """A rows x cols box has a one-round resident plan (all tiles co-resident)."""
    return resident_shape(rows, cols, depth) is not None


RES_MIN_PASSES = 4  # csrc/include/heat/plan.hpp kResMinPasses


def _blocks(n: int, parts: int) -> List[int]:
    """Remainder-aware 1-D block sizes (topology.cpp block_span)."""
    return [n // parts + (1 if i < n % parts else 0) for i in range(parts)]


def resident_halo_passes(nx: int, ny: int, px: int, py: int, depth: int = 12,
                         mmax: int = 8) -> int:
    """The solver's resident-aware passes per exchange (topology.cpp
    resident_halo_passes): the largest m in [2, mmax] for which every rank's
    first span box -- the owned block grown by (m - 1) * depth on each side
    with a neighbour -- has a one-round resident plan of the same tile shape
    as its owned block's; 0 if the owned blocks have none or no m keeps it.
    The solver keeps m = 8 below RES_MIN_PASSES."""
    if px * py < 2:
        return 0
    rows, cols = _blocks(nx, px), _blocks(ny, py)
    own = {(r, c): resident_shape(r, c, depth) for r in rows for c in cols}
    if any(v is None for v in own.values()):
        return 0
    ext = min((rows if px > 1 else []) + (cols if py > 1 else []))
    for m in range(min(mmax, ext // depth), 1, -1):
        gr = (m - 1) * depth if px > 1 else 0
        gc = ((m - 1) * depth) // 4 * 4 if py > 1 else 0
        ok = True
        for i, r in enumerate(rows):
            for j, c in enumerate(cols):
                er = gr * ((i > 0) + (i < px - 1))
                ec = gc * ((j > 0) + (j < py - 1))
                ok = ok and resident_shape(r + er, c + ec, depth) == own[(r, c)]
        if ok:
            return m
    return 0


def _interp(pts, srps: float) -> float:
    if srps <= pts[0][0]:
        return pts[0][1] * srps / pts[0][0] if srps > 0 else pts[0][1]
    for (x0, y0), (x1, y1) in zip(pts, pts[1:]):
        if srps <= x1:
            return y0 + (y1 - y0) * (srps - x0) / (x1 - x0)
    return pts[-1][1]


def rate_tcells(rows: int, cols: int, resident: bool = None) -> float:
    """Interpolated whole-solver rate of a rows x cols block (Tcells/s);
    `resident` (default: whether the block itself fits one round) picks the
    family."""
    srps = math.ceil(cols / STRIP_COLS) * rows / SIMDS
    if resident is None:
        resident = resident_fits(rows, cols)
    return _interp(RESIDENT_POINTS if resident else STREAM_POINTS, srps)


def _grid(cfg: HeatConfig, world: int) -> tuple:
    if cfg.px > 0 and cfg.py > 0:
        return cfg.px, cfg.py
    if cfg.decomp in ("rows", "1d"):
        return world, 1
    d = dims_create(world, 2)
    return d[0], d[1]


# A fit is trusted (and may prune autotune candidates) only with at least
# FIT_MIN_SIZES distinct message sizes, a positive slope and an R^2 of at
# least FIT_MIN_R2 over the per-size medians.
FIT_MIN_SIZES = 3
FIT_MIN_R2 = 0.8


def fit_exchange(points: Sequence[tuple], base: Dict = None) -> Dict:
    """Exchange parameters from measured (message bytes, seconds per grouped
    exchange) samples on the real ranks (``HeatSolver.time_exchange``, max
    over ranks; several samples per size allowed): the median per size, then
    latency = intercept and link_gbps = 1 / slope of a least-squares line.

    Returns a copy of `base` (default XGMI) with ``fit_ok`` and the medians
    attached.  Only a trustworthy fit (>= FIT_MIN_SIZES sizes, slope > 0,
    intercept >= 0, R^2 >= FIT_MIN_R2) replaces the stated latency and
    bandwidth; otherwise ``fit_ok`` is False, the stated values stay and
    ``prune`` keeps every candidate (round 5's 8-rank rehearsal fitted a
    negative slope from two noisy points and set the latency to 20.6 ms,
    which pruned four candidates untimed)."""
    out = dict(base or XGMI)
    by_size: Dict[float, List[float]] = {}
    for b, t in points:
        if t > 0:
            by_size.setdefault(float(b), []).append(float(t))
    med = sorted((b, sorted(ts)[len(ts) // 2] if len(ts) % 2 else
                  0.5 * (sorted(ts)[len(ts) // 2 - 1] + sorted(ts)[len(ts) // 2]))
                 for b, ts in by_size.items())
    out["measured"] = [[int(b), round(t * 1e6, 3)] for b, t in med]
    out["fit_ok"] = False
    if len(med) < 2:
        out["fit_reason"] = f"{len(med)} message size(s)"
        return out
    n = len(med)
    mb = sum(b for b, _ in med) / n
    mt = sum(t for _, t in med) / n
    sxx = sum((b - mb) ** 2 for b, _ in med)
    syy = sum((t - mt) ** 2 for _, t in med)
    sxy = sum((b - mb) * (t - mt) for b, t in med)
    slope = sxy / sxx
    lat = mt - slope * mb
    r2 = (sxy * sxy / (sxx * syy)) if syy > 0 else 1.0
    out["fit_r2"] = round(r2, 4)
    if n < FIT_MIN_SIZES:
        out["fit_reason"] = f"{n} message sizes (< {FIT_MIN_SIZES})"
    elif slope <= 0:
        out["fit_reason"] = "non-positive slope"
    elif lat < 0:
        out["fit_reason"] = "negative latency"
    elif r2 < FIT_MIN_R2:
        out["fit_reason"] = f"R^2 {r2:.3f} < {FIT_MIN_R2}"
    else:
        out["fit_ok"] = True
        out["link_gbps"] = round(1.0 / slope / 1e9, 3)
        out["latency_us"] = round(lat * 1e6, 3)
    return out


def predict(cfg: HeatConfig, world: int, depth: int = 12, halo_passes: int = 8,
            xgmi: Dict = None) -> Dict:
    """Predicted time per 1000 iterations and node throughput of cfg on
    `world` GPUs (the slowest rank: the largest block, with neighbours).
    `xgmi`: exchange parameters (default the stated XGMI; fit_exchange gives
    measured ones)."""
    X = xgmi or XGMI
    px, py = _grid(cfg, world)
    lx = math.ceil(cfg.nx / px)
    ly = math.ceil(cfg.ny / py)
    m = cfg.halo_passes or halo_passes
    if not cfg.halo_passes and world > 1:
        rm = resident_halo_passes(cfg.nx, cfg.ny, px, py, depth)
        if rm >= RES_MIN_PASSES:
            m = rm
    if world == 1:
        m = 1
    schedule = cfg.schedule if cfg.schedule != "auto" else "sync"
    if world > 1 and schedule != "sync":
        m = 1
    H = m * depth
    # Deep-halo ghost rows recomputed on the decomposed axes: the first
    # pass's box (resident launches keep it for all m passes) grows by H - K
    # per neighbour side, two for an inner rank (p > 2), one with p = 2.
    ext_r = (2 if px > 2 else 1) * (H - depth) if px > 1 else 0
    ext_c = (2 if py > 2 else 1) * (H - depth) if py > 1 else 0
    resident = schedule == "sync" and resident_fits(lx + ext_r, ly + ext_c, depth)
    if resident:
        # The span box's long-span rate, less the span's load / store.
        rate = rate_tcells(lx + ext_r, ly + ext_c, True) * 1e12
        if world > 1:
            rate /= 1.0 + SPAN_COST / m
    else:
        rate = rate_tcells(lx, ly, False) * 1e12
    cells = (lx + ext_r) * (ly + ext_c)
    compute_s = cells * 1000 / rate
    exchanges = math.ceil(1000 / H) if world > 1 else 0
    ns_bytes = H * (ly + 2 * H) * 4 if px > 1 else 0
    ew_bytes = lx * H * 4 if py > 1 else 0
    msg = max(ns_bytes, ew_bytes)
    t_ex = (X["latency_us"] * 1e-6 + msg / (X["link_gbps"] * 1e9) +
            (2 * X["pack_us"] * 1e-6 if py > 1 else 0.0))
    ex_total = exchanges * t_ex
    if schedule != "sync" and world > 1:
        # Overlap schedules: one K-deep exchange per pass, hidden behind the
        # interior launch, but the boundary bands are separate latency-bound
        # launches and every pass pays a cross-stream join (~10-15 us each,
        # profiles/overlap_probe_r1.md); no resident spans (split kernels).
        passes = math.ceil(1000 / depth)
        per_pass = lx * ly * depth / (rate_tcells(lx, ly, False) * 1e12 * 0.8)
        compute_s = passes * (max(per_pass, t_ex) + 25e-6)
        ex_total = 0.0
    checks = math.floor(1000 / cfg.check_interval) if cfg.converge else 0
    reduce_s = checks * X["allreduce_us"] * 1e-6 if world > 1 else 0.0
    total = compute_s + ex_total + reduce_s
    return {
        "layout": f"{px}x{py}", "block": f"{lx}x{ly}", "schedule": schedule,
        "halo": H, "exchanges_per_1000": exchanges,
        "compute_ms": round(compute_s * 1e3, 4),
        "exchange_ms": round(ex_total * 1e3, 4),
        "reduce_ms": round(reduce_s * 1e3, 4),
        "ms_per_1000": round(total * 1e3, 4),
        "tcells_per_s": round(cfg.nx * cfg.ny * 1000 / total / 1e12, 3),
        "rank_rate_tcells": round(rate / 1e12, 3),
        "resident": bool(resident) if schedule == "sync" else False,
        "message_bytes": msg,
    }


def prune(cands: Sequence[HeatConfig], world: int, slack: float = 1.3,
          xgmi: Dict = None) -> List[HeatConfig]:
    """The candidates the autotune times: those whose predicted time is
    within `slack` x the best prediction, plus the best-predicted candidate
    of every (layout, passes per exchange) pair, so a model error can cost a
    schedule but never a whole layout or halo depth.  With a measured
    exchange fit that failed its quality checks (``xgmi["fit_ok"]`` False)
    nothing is pruned."""
    if len(cands) <= 1 or (xgmi is not None and not xgmi.get("fit_ok", True)):
        return list(cands)
    t = [predict(c, world, xgmi=xgmi)["ms_per_1000"] for c in cands]
    best = min(t)
    group_best: Dict[tuple, float] = {}
    for c, x in zip(cands, t):
        k = (_grid(c, world), c.halo_passes)
        group_best[k] = min(group_best.get(k, float("inf")), x)
    return [c for c, x in zip(cands, t)
            if x <= slack * best or x == group_best[(_grid(c, world), c.halo_passes)]]


def model_params(xgmi: Dict = None) -> Dict:
    return {"xgmi": dict(xgmi or XGMI), "resident_points": [list(p) for p in RESIDENT_POINTS],
            "span_cost": SPAN_COST,
            "stream_points": [list(p) for p in STREAM_POINTS],
            "strip_cols": STRIP_COLS, "simds": SIMDS}
