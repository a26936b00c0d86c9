"""The TB launch-planner knobs (heat::gpu::TbTuning) and variant flags as a
named API instead of process-global environment variables (no GPU needed)."""
import pytest

from parallel_heat_amd import ops


def test_tuning_roundtrip():
    saved = ops.tb_tuning()
    try:
        t = ops.TbTuning(variant=int(ops.TbVariant.DEFAULT), rounds=2, min_len=24, waves=512,
                         edge_frac=0.75, age_weights=[1.5, 1.0], tile_rows=16, tile_waves=8, nt=1)
        ops.set_tb_tuning(t)
        assert ops.tb_tuning() == t
        with pytest.raises(ValueError):
            ops.set_tb_tuning(ops.TbTuning(age_weights=[1.0] * 5))
    finally:
        ops.set_tb_tuning(saved)
    assert ops.tb_tuning() == saved


def test_variant_flags_match_the_engine():
    V = ops.TbVariant
    assert int(V.DEFAULT) == 23 and int(V.DEFAULT_DEEP) == 2071
    assert V.DEFAULT_DEEP & V.SPLIT and V.DEFAULT & V.SCALAR and (V.DEFAULT & 3) == V.RAMP
    # csrc/include/heat/kernels.hpp tbv:: values
    import re
    from parallel_heat_amd import _native
    src = (_native.REPO_DIR / "csrc" / "include" / "heat" / "kernels.hpp").read_text()
    names = {"kRing3": V.RING3, "kRing4": V.RING4, "kRing2": V.RING2, "kRamp": V.RAMP,
             "kScalar": V.SCALAR, "kXcdGroups": V.XCD_GROUPS, "kAltDirection": V.ALT_DIRECTION,
             "kFloat2": V.FLOAT2, "kForceAgePairs": V.FORCE_AGE_PAIRS, "kSplit": V.SPLIT,
             "kDiagNoStore": V.DIAG_NO_STORE, "kDiagCachedRows": V.DIAG_CACHED_ROWS,
             "kNoAgePairs": V.NO_AGE_PAIRS, "kLinear": V.LINEAR, "kNoLinear": V.NO_LINEAR,
             "kTile": V.TILE, "kTileDpp": V.TILE_DPP}
    for n, v in names.items():
        m = re.search(rf"\b{n} = (\d+),", src)
        assert m and int(m.group(1)) == int(v), n
