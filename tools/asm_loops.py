#!/usr/bin/env python3
"""Instruction mix of the loops of one kernel in a `make asm` listing.

    python tools/asm_loops.py build/asm/tb_split.s tb_split_kernelILi12ELi6E [--min 100]

With --scratch, the number of scratch (spill / reload) instructions per loop
instead: a spill outside every step loop costs little, one inside costs a
memory round trip per iteration (tests/test_kernel_resources.py, the budget).

A loop is a backward branch (s_cbranch_* / s_branch to an earlier label); its
body is the text from the target label to the branch.  For each loop with at
least --min instructions it prints the count per class (VALU arithmetic, DPP,
moves, v_cndmask, LDS, global memory, SALU, waits, branches, other) so the
non-arithmetic share of a hot loop is visible without a GPU.
"""
import argparse
import collections
import re


def classify(op, line):
    if op.startswith("s_waitcnt") or op == "s_nop" or op == "s_sleep":
        return "wait"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("v_"):
        if "dpp" in line or "row_" in line or "wave_sh" in line:
            return "valu_dpp"
        if op.startswith(("v_fma", "v_fmac", "v_add_f32", "v_sub_f32", "v_pk_fma", "v_pk_add",
                          "v_mul_f32")):
            return "valu_fp"
        if op.startswith("v_mov") or op.startswith("v_accvgpr"):
            return "valu_mov"
        if op.startswith("v_cndmask"):
            return "valu_cndmask"
        return "valu_other"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel", help="substring of the mangled kernel name")
    ap.add_argument("--min", type=int, default=100)
    ap.add_argument("--other", action="store_true", help="list the valu_other opcodes")
    ap.add_argument("--scratch", action="store_true",
                    help="only print the scratch (spill / reload) instructions inside each loop "
                         "and in the whole kernel")
    a = ap.parse_args()
    lines = open(a.asm).read().splitlines()
    start = next(i for i, l in enumerate(lines)
                 if re.match(r"^_Z\S*:", l) and a.kernel in l.split(":")[0])
    end = next((i for i in range(start + 1, len(lines)) if re.match(r"^_Z\S*:", lines[i])),
               len(lines))
    body = lines[start:end]
    if a.scratch:
        print(f"scratch instructions in the kernel: {sum('scratch_' in l for l in body)}")
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.match(r"^\s+(s_cbranch_\w+|s_branch)\s+(\.LBB\w+)", l)
        if not m or m.group(2) not in labels or labels[m.group(2)] >= i:
            continue
        cnt = collections.Counter()
        others = collections.Counter()
        for l2 in body[labels[m.group(2)]:i + 1]:
            s = l2.strip()
            if not s or s.startswith((";", ".")) or s.endswith(":"):
                continue
            op = s.split()[0]
            c = classify(op, s)
            cnt[c] += 1
            if c == "valu_other":
                others[op] += 1
        n = sum(cnt.values())
        if n < a.min:
            continue
        if a.scratch:
            sc = sum(1 for l2 in body[labels[m.group(2)]:i + 1] if "scratch_" in l2)
            print(f"loop {m.group(2)} (lines {start + labels[m.group(2)] + 1}-{start + i + 1}): "
                  f"{n} instrs, {sc} scratch")
            continue
        print(f"loop {m.group(2)} (lines {start + labels[m.group(2)] + 1}-{start + i + 1}): {n} instrs")
        for k, v in sorted(cnt.items(), key=lambda kv: -kv[1]):
            print(f"  {k:14s} {v}")
        if a.other and others:
            print("  other ops:", dict(others.most_common(12)))


if __name__ == "__main__":
    main()
