"""Tensor-level access to the native stencil kernels.

These wrap single kernels of ``csrc/kernels/stencil.hip`` for torch tensors
(device kernels on ROCm tensors, the OpenMP oracle on CPU tensors), so the
kernels can be tested against plain PyTorch fp32 and composed into custom
schedules.  Fields use the engine's memory layout (ghost ring + 256-B pitch,
``heat::Layout``); ``Field`` owns a torch tensor with that layout.

Reference kernels: ``heat`` (``cuda/cuda_heat.cu:140-163``) and the fused
``heat<threads>`` + ``semi_reduce`` residual (``:32-138``).
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import torch

from .. import _native
from ..models.config import INIT_MODES
from ..parallel.topology import layout

Box = Tuple[int, int, int, int]  # (r0, r1, c0, c1) in local coordinates


class TbVariant(enum.IntFlag):
    """Variant flags of the temporally blocked kernel (``heat::gpu::tbv`` in
    csrc/include/heat/kernels.hpp).  The low two bits pick the register
    pipeline; the rest pick the build and the launch layout."""
    RING3 = 0             # 3-row rings, skew 1
    RING4 = 1             # 4-row rings, skew 2
    RING2 = 2             # 2-row rings + copy
    RAMP = 3              # 3-row rings + compile-time ramp skip
    SCALAR = 4            # scalar row-update build (depth 12 lives here)
    XCD_GROUPS = 16       # contiguous wave ranges per XCD
    ALT_DIRECTION = 32    # odd chunks stream bottom-up
    FLOAT2 = 64           # float2 lanes (128-column strips)
    FORCE_AGE_PAIRS = 256  # age groups even at equal weights
    DIAG_NO_STORE = 1024  # diagnostics: no output stores (wrong results)
    SPLIT = 2048          # two-wave level-split pipelines (depths 8, 12)
    DIAG_CACHED_ROWS = 4096  # diagnostics: cache-resident input rows (wrong results)
    NO_AGE_PAIRS = 16384  # never age-group
    LINEAR = 32768        # force the balanced plan: equal strip-rows per unit
    NO_LINEAR = 65536     # never switch to it (default: when the classic plan fills < 90 %)
    TILE = 131072         # workgroup tiles: 8 waves x R rows in VGPRs, LDS row exchange per step
    TILE_DPP = 262144     # with TILE: DPP lane shifts instead of ds_bpermute
    SHIFT_MIXED = 524288  # with SPLIT: west shift DPP, east ds_bpermute (tb_split_mixed.hip)
    DEFAULT = RAMP | SCALAR | XCD_GROUPS       # 23
    DEFAULT_DEEP = DEFAULT | SPLIT             # 2071


@dataclass
class TbTuning:
    """Launch-planner knobs (``heat::gpu::TbTuning``); HEAT_TB_* environment
    variables seed them when the library is first used."""
    variant: int = -1
    rounds: int = 0
    min_len: int = 0
    waves: int = 0
    edge_frac: float = 1.0
    age_weights: List[float] = field(default_factory=list)
    tile_rows: int = 0  # rows per wave of TILE launches (0: planner)
    tile_waves: int = 0  # waves per TILE workgroup, 8 or 16 (0: planner)
    tile_xl: int = -1  # TILE lane shifts: 0 DPP, 1 ds_bpermute, 2 mixed (-1: default)
    nt: int = -1  # level-split rows non-temporal 1 / plain 0 (-1: by the bytes a pass sweeps)


def tb_tuning() -> TbTuning:
    t = _native.HeatTbTuning()
    _native.call("heat_tb_get_tuning", ctypes.byref(t))
    return TbTuning(t.variant, t.rounds, t.min_len, t.waves, t.edge_frac,
                    [t.weights[i] for i in range(t.n_weights)], t.tile_rows, t.tile_waves,
                    t.tile_xl, t.nt)


def set_tb_tuning(t: TbTuning) -> None:
    n = len(t.age_weights)
    if n > 4:
        raise ValueError("at most 4 age weights")
    c = _native.HeatTbTuning(int(t.variant), int(t.rounds), int(t.min_len), int(t.waves),
                             float(t.edge_frac), n, int(t.tile_rows),
                             (ctypes.c_double * 4)(*t.age_weights), int(t.tile_waves),
                             int(t.tile_xl), int(t.nt), 0)
    _native.call("heat_tb_set_tuning", ctypes.byref(c))


@dataclass
class Geom:
    """Global placement of a local field: local (0,0) is global (gx0, gy0)."""
    nx: int
    ny: int
    gx0: int = 0
    gy0: int = 0
    cx: float = 0.1
    cy: float = 0.1


class Field:
    """A local field (owned lx x ly block + `halo`-deep ghost ring) in a torch tensor."""

    def __init__(self, lx: int, ly: int, halo: int = 1, device="cpu", fill: float = 0.0):
        self.lx, self.ly, self.halo = lx, ly, halo
        self.pitch, self.rows, self.hx, self.hy = layout(lx, ly, halo)
        self.data = torch.full((self.rows, self.pitch), fill, dtype=torch.float32,
                               device=device)

    @property
    def device(self):
        return self.data.device

    def ptr(self) -> int:
        """Address of owned cell (0, 0)."""
        return self.data.data_ptr() + 4 * (self.hx * self.pitch + self.hy)

    def view(self, r0: int, r1: int, c0: int, c1: int) -> torch.Tensor:
        """View of local cells [r0,r1) x [c0,c1) (negative = ghost ring)."""
        return self.data[self.hx + r0:self.hx + r1, self.hy + c0:self.hy + c1]

    def owned(self) -> torch.Tensor:
        return self.view(0, self.lx, 0, self.ly)

    def set_owned(self, t: torch.Tensor) -> None:
        self.owned().copy_(t)


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream if torch.cuda.is_available() else 0


def _resid_ptr(resid: Optional[torch.Tensor]) -> Optional[int]:
    if resid is None:
        return None
    if resid.dtype != torch.int32 or resid.numel() < 1:
        raise ValueError("resid must be an int32 tensor (float bits of max|delta|)")
    return resid.data_ptr()


def resid_value(resid: torch.Tensor) -> float:
    """Decode the float bits an atomic-max residual word holds."""
    return float(resid[:1].cpu().view(torch.float32).item())


def init_field(f: Field, geom: Geom, mode: str = "ref-wrap", seed: int = 0) -> None:
    """Fill every cell of the field (owned, ghosts, padding) from the initial condition."""
    m = INIT_MODES[mode]
    if f.device.type == "cpu":
        from ..models.reference import init_grid
        full = init_grid(geom.nx, geom.ny, mode, seed)  # small fields only
        f.data.zero_()
        r0, r1 = max(0, geom.gx0 - f.hx), min(geom.nx, geom.gx0 + f.lx + f.hx)
        c0, c1 = max(0, geom.gy0 - f.hy), min(geom.ny, geom.gy0 + f.pitch - f.hy)
        f.data[r0 - geom.gx0 + f.hx:r1 - geom.gx0 + f.hx, c0 - geom.gy0 + f.hy:c1 - geom.gy0 + f.hy] = \
            torch.from_numpy(full[r0:r1, c0:c1])
        return
    _native.call("heat_op_init", ctypes.c_void_p(f.ptr()), f.lx, f.ly, f.halo, geom.gx0,
                 geom.gy0, geom.nx, geom.ny, m, seed, ctypes.c_void_p(_stream()))


def naive_step(src: Field, dst: Field, geom: Geom, box: Optional[Box] = None,
               resid: Optional[torch.Tensor] = None) -> None:
    """One Jacobi step over `box` (default: the owned block)."""
    r0, r1, c0, c1 = box or (0, src.lx, 0, src.ly)
    if src.pitch != dst.pitch:
        raise ValueError("src/dst layouts differ")
    if src.device.type == "cpu":
        r = ctypes.c_float()
        _native.call("heat_cpu_step", ctypes.c_void_p(src.ptr()), ctypes.c_void_p(dst.ptr()),
                     src.pitch, geom.gx0, geom.gy0, geom.nx, geom.ny, geom.cx, geom.cy,
                     r0, r1, c0, c1, ctypes.byref(r) if resid is not None else None)
        if resid is not None:
            resid.view(torch.float32)[0] = max(resid_value(resid), r.value)
        return
    rp = _resid_ptr(resid)
    _native.call("heat_op_naive_step", ctypes.c_void_p(src.ptr()), ctypes.c_void_p(dst.ptr()),
                 src.pitch, geom.gx0, geom.gy0, geom.nx, geom.ny, geom.cx, geom.cy,
                 r0, r1, c0, c1, ctypes.c_void_p(rp) if rp else None,
                 ctypes.c_void_p(_stream()))


def lds_step(src: Field, dst: Field, geom: Geom, box: Optional[Box] = None,
             resid: Optional[torch.Tensor] = None, numerics: str = "fp32") -> None:
    """One Jacobi step over `box` with the LDS-staged tile kernel (GPU only);
    numerics "fp32" (canonical FMA) or "mpi" (reference MPI double arithmetic)."""
    r0, r1, c0, c1 = box or (0, src.lx, 0, src.ly)
    if src.pitch != dst.pitch:
        raise ValueError("src/dst layouts differ")
    if src.device.type != "cuda":
        raise ValueError("lds_step needs GPU fields")
    rp = _resid_ptr(resid)
    _native.call("heat_op_lds_step", ctypes.c_void_p(src.ptr()), ctypes.c_void_p(dst.ptr()),
                 src.pitch, geom.gx0, geom.gy0, geom.nx, geom.ny, geom.cx, geom.cy,
                 r0, r1, c0, c1, ctypes.c_void_p(rp) if rp else None,
                 ctypes.c_void_p(_stream()), {"fp32": 0, "mpi": 1}[numerics])


def mfma_step(src: Field, dst: Field, geom: Geom, box: Optional[Box] = None,
              resid: Optional[torch.Tensor] = None) -> None:
    """One Jacobi step over `box` as banded matmuls on the fp32 MFMA units
    (GPU only; rounding differs from the canonical expression by ~1 ulp)."""
    r0, r1, c0, c1 = box or (0, src.lx, 0, src.ly)
    if src.pitch != dst.pitch:
        raise ValueError("src/dst layouts differ")
    if src.device.type != "cuda":
        raise ValueError("mfma_step needs GPU fields")
    rp = _resid_ptr(resid)
    _native.call("heat_op_mfma_step", ctypes.c_void_p(src.ptr()), ctypes.c_void_p(dst.ptr()),
                 src.pitch, geom.gx0, geom.gy0, geom.nx, geom.ny, geom.cx, geom.cy,
                 r0, r1, c0, c1, ctypes.c_void_p(rp) if rp else None,
                 ctypes.c_void_p(_stream()))


def tb_step(src: Field, dst: Field, geom: Geom, depth: int,
            boxes: Optional[Sequence[Box]] = None, resid: Optional[torch.Tensor] = None,
            waves_target: int = 0, variant: int = -1, res_level: int = 0) -> None:
    """`depth` fused Jacobi steps (temporally blocked kernel) over up to 5 boxes.

    variant: -1 = chosen per launch (TbVariant.DEFAULT, or DEFAULT_DEEP for
    large depth-12 launches); otherwise TbVariant flags.  res_level (with
    resid): the step 1..depth whose max |new - old| goes to resid (0 = the
    last; inner levels need tb_mid_residual(depth)).
    """
    if src.device.type == "cpu":
        raise ValueError("tb_step is a GPU kernel")
    if not _native.lib().heat_tb_supported(depth):
        raise ValueError(f"unsupported depth {depth}")
    if src.halo < depth or src.hy < -(-depth // 4) * 4:
        raise ValueError("ghost ring thinner than depth")
    boxes = list(boxes or [(0, src.lx, 0, src.ly)])
    arr = (ctypes.c_int64 * (4 * len(boxes)))(*[v for b in boxes for v in b])
    rp = _resid_ptr(resid)
    _native.call("heat_op_tb_step", ctypes.c_void_p(src.ptr()), ctypes.c_void_p(dst.ptr()),
                 src.pitch, geom.gx0, geom.gy0, geom.nx, geom.ny, geom.cx, geom.cy, arr,
                 len(boxes), depth, ctypes.c_void_p(rp) if rp else None,
                 ctypes.c_void_p(_stream()), waves_target, int(variant), int(res_level))


def tb_stamps(buf: Optional[torch.Tensor]) -> None:
    """Diagnostics: record per-wave clock stamps of the following tb_step
    launches into `buf` (int64 GPU tensor, 4 per wave: start, end in 100 MHz
    ticks, block, strip << 32 | chunk); None switches recording off."""
    if buf is None:
        _native.call("heat_op_tb_stamps", None, 0)
        return
    if buf.dtype != torch.int64 or buf.device.type != "cuda":
        raise ValueError("stamps need an int64 GPU tensor")
    _native.call("heat_op_tb_stamps", ctypes.c_void_p(buf.data_ptr()), buf.numel() // 4)


def pack(f: Field, box: Box, out: torch.Tensor) -> None:
    r0, r1, c0, c1 = box
    if f.device.type == "cpu":
        out.view(r1 - r0, c1 - c0).copy_(f.view(r0, r1, c0, c1))
        return
    _native.call("heat_op_pack", ctypes.c_void_p(f.ptr()), f.pitch, r0, r1, c0, c1,
                 ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(_stream()))


def unpack(buf: torch.Tensor, f: Field, box: Box) -> None:
    r0, r1, c0, c1 = box
    if f.device.type == "cpu":
        f.view(r0, r1, c0, c1).copy_(buf.view(r1 - r0, c1 - c0))
        return
    _native.call("heat_op_unpack", ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(f.ptr()),
                 f.pitch, r0, r1, c0, c1, ctypes.c_void_p(_stream()))


def residual(a: Field, b: Field, box: Optional[Box] = None,
             resid: Optional[torch.Tensor] = None) -> float:
    """max |a - b| over `box` (owned block by default)."""
    r0, r1, c0, c1 = box or (0, a.lx, 0, a.ly)
    if a.device.type == "cpu":
        return float((a.view(r0, r1, c0, c1) - b.view(r0, r1, c0, c1)).abs().max())
    own = resid is None
    if own:
        resid = torch.zeros(1, dtype=torch.int32, device=a.device)
    _native.call("heat_op_residual", ctypes.c_void_p(a.ptr()), ctypes.c_void_p(b.ptr()),
                 a.pitch, r0, r1, c0, c1, ctypes.c_void_p(resid.data_ptr()),
                 ctypes.c_void_p(_stream()))
    return resid_value(resid) if own else float("nan")
