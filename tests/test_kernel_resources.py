"""Spill guardrail (the reference's equivalent is the
`--ptxas-options=-v` resource report of /root/reference/cuda/Makefile:5).

The built libheat.so's gfx950 code-object metadata (tools/kernel_resources.py,
no GPU needed) is checked against tests/data/kernel_scratch_budget.json:

* every kernel of the hot families (level-split and streaming TB kernels,
  workgroup tiles, resident tiles) must stay at or below its recorded scratch
  bytes per lane -- a ratchet: an edit that makes a kernel spill more fails;
* the instantiations the default 1-8 GPU paths run in their main loops
  without checks (resident tiles and tile passes, RES 0, every shape and lane
  shift) must have NO scratch at all;
* a hot kernel missing from the budget must have no scratch either.

Kernels that do spill keep it outside their step loops (checked from the ISA
with tools/asm_loops.py --scratch; profiles/r5_spills.md lists them).
Regenerate the budget after an intended change with
`python tools/kernel_resources.py --budget > tests/data/kernel_scratch_budget.json`.
"""
import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "parallel_heat_amd", "_lib", "libheat.so")
BUDGET = os.path.join(ROOT, "tests", "data", "kernel_scratch_budget.json")

# Namespaces of the hot kernel families (tbp / tbn: diagnostic variants).
HOT = re.compile(r"^_ZN4heat3gpu(3tbx|4tbxm|4tbxn|3tbc|3tbs|3tbw)")
# Must be spill-free: the tile passes (with or without residuals, since
# round 5's branch-free last-step stores), default (mixed) lane shifts XL 2.
# Exempt: 20 x 16 RES 1 (12 B/lane).  The unchecked resident launches may
# keep at most 32 B/lane of pass-level state in scratch (20 x 16, and the
# packed-update 12-row shapes: 1-2 scratch instructions per pass, none in
# the step loops, profiles/r5_spills.md); the budget holds each at its value.
ZERO = re.compile(r"tbw11tile_kernelILi\d+ELi\d+ELi2ELi[01]E")
ZERO_EXEMPT = re.compile(r"ILi20ELi16E")
SMALL = re.compile(r"tbw20tile_resident_kernelILi\d+ELi\d+ELi2ELi0E")


def _kernels():
    if not os.path.exists(LIB):
        pytest.skip("libheat.so not built")
    from kernel_resources import kernels
    try:
        return kernels(LIB)
    except (OSError, Exception) as e:  # noqa: BLE001 - toolchain missing
        pytest.skip(f"cannot read code objects: {e}")


def test_hot_kernels_within_scratch_budget():
    ks = [k for k in _kernels() if HOT.match(k["name"])]
    assert len(ks) >= 60, len(ks)
    budget = json.load(open(BUDGET))
    over = [(k["name"], k["scratch"], budget.get(k["name"], 0)) for k in ks
            if k["scratch"] > budget.get(k["name"], 0)]
    assert not over, "kernels spill more than their budget: %r" % over


def test_default_tile_paths_spill_free():
    ks = [k for k in _kernels() if ZERO.search(k["name"]) and not ZERO_EXEMPT.search(k["name"])]
    assert len(ks) >= 16, len(ks)
    bad = [(k["name"], k["scratch"], k["vgpr"]) for k in ks if k["scratch"] > 0]
    assert not bad, "default tile instantiations spill: %r" % bad
    rs = [k for k in _kernels() if SMALL.search(k["name"])]
    assert len(rs) >= 8, len(rs)
    bad = [(k["name"], k["scratch"]) for k in rs if k["scratch"] > 32]
    assert not bad, "unchecked resident instantiations spill more than 32 B/lane: %r" % bad
