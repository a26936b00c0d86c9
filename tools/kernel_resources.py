#!/usr/bin/env python3
"""Per-kernel register / scratch report of a built libheat.so (gfx950).

    python tools/kernel_resources.py [parallel_heat_amd/_lib/libheat.so] [--spills] [--json]

Reads the AMDGPU code-object metadata the compiler wrote into the library
(the same numbers `-Rpass-analysis=kernel-resource-usage` prints, and what
the reference's `--ptxas-options=-v` reported for its CUDA kernels,
/root/reference/cuda/Makefile:5): VGPRs, AGPRs, SGPRs, scratch bytes per lane
(`private_segment_fixed_size`) and spilled VGPRs, for every kernel of every
compilation unit.  No GPU needed: the gfx950 code objects are unbundled with
llvm-objdump --offloading into a temporary directory and read with
llvm-readelf --notes.  `make resources` runs it; tests/test_kernel_resources.py
fails when a hot kernel grows scratch.
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
LLVM = os.path.join(ROCM, "llvm", "bin")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(ROOT, "parallel_heat_amd", "_lib", "libheat.so")

_FIELDS = ("name", "private_segment_fixed_size", "vgpr_count", "agpr_count", "sgpr_count",
           "vgpr_spill_count", "sgpr_spill_count", "group_segment_fixed_size")
_LINE = re.compile(r"^\s*(?:- )?\.(%s):\s+(\S+)" % "|".join(_FIELDS))


def _demangle(names):
    try:
        p = subprocess.run([os.path.join(LLVM, "llvm-cxxfilt")], input="\n".join(names),
                           capture_output=True, text=True, check=True)
        out = p.stdout.splitlines()
        if len(out) == len(names):
            return out
    except (OSError, subprocess.CalledProcessError):
        pass
    return list(names)


def kernels(lib=DEFAULT_LIB):
    """One dict per kernel: name (mangled), pretty, scratch, vgpr, agpr, sgpr,
    vgpr_spill, sgpr_spill, lds, unit (code-object index)."""
    out = []
    with tempfile.TemporaryDirectory() as d:
        # --offloading writes the bundles next to its input: work on a copy.
        copy = os.path.join(d, "lib.so")
        shutil.copyfile(lib, copy)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", copy],
                       capture_output=True, text=True, check=True)
        objs = sorted(f for f in os.listdir(d) if f.endswith("gfx950"))
        for unit, f in enumerate(objs):
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes",
                                    os.path.join(d, f)],
                                   capture_output=True, text=True, check=True).stdout
            cur = None
            for line in notes.splitlines():
                m = _LINE.match(line)
                if not m:
                    continue
                key, val = m.group(1), m.group(2)
                if line.lstrip().startswith("- "):
                    cur = {"unit": unit}
                    out.append(cur)
                if cur is None:
                    continue
                cur[key] = val if key == "name" else int(val)
    out = [k for k in out if "name" in k]
    pretty = _demangle([k["name"] for k in out])
    res = []
    for k, p in zip(out, pretty):
        res.append({"name": k["name"], "pretty": p, "unit": k["unit"],
                    "scratch": k.get("private_segment_fixed_size", 0),
                    "vgpr": k.get("vgpr_count", 0), "agpr": k.get("agpr_count", 0),
                    "sgpr": k.get("sgpr_count", 0), "vgpr_spill": k.get("vgpr_spill_count", 0),
                    "sgpr_spill": k.get("sgpr_spill_count", 0),
                    "lds": k.get("group_segment_fixed_size", 0)})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=DEFAULT_LIB)
    ap.add_argument("--spills", action="store_true", help="only kernels with scratch > 0")
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--budget", action="store_true",
                    help="JSON {kernel: scratch bytes} of the hot families "
                         "(tests/data/kernel_scratch_budget.json)")
    a = ap.parse_args()
    ks = kernels(a.lib)
    if a.budget:
        hot = re.compile(r"^_ZN4heat3gpu(3tbx|4tbxm|4tbxn|3tbc|3tbs|3tbw)")
        print(json.dumps({k["name"]: k["scratch"] for k in sorted(ks, key=lambda k: k["name"])
                          if hot.match(k["name"]) and k["scratch"] > 0}, indent=1))
        return 0
    if a.spills:
        ks = [k for k in ks if k["scratch"] > 0 or k["vgpr_spill"] > 0]
    if a.json:
        print(json.dumps(ks, indent=1))
        return 0
    print(f"{'vgpr':>4} {'agpr':>4} {'sgpr':>4} {'scratch':>7} {'spill':>5} {'lds':>6}  kernel")
    for k in sorted(ks, key=lambda k: k["pretty"]):
        print(f"{k['vgpr']:4d} {k['agpr']:4d} {k['sgpr']:4d} {k['scratch']:7d} "
              f"{k['vgpr_spill']:5d} {k['lds']:6d}  {k['pretty'][:150]}")
    print(f"{len(ks)} kernels", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
