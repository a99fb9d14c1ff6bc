#!/usr/bin/env python3
"""Instruction mix of a kernel's loops from device assembly (``hipcc --cuda-device-only -S``).

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast --cuda-device-only -S csrc/attention.hip -o /tmp/attn.s
  python scripts/isa_loop_stats.py /tmp/attn.s attn_bwd_kernelILi64ELb0E

For every backward branch (a loop: ``s_cbranch_* / s_branch`` to an earlier label) prints the span's
counts of MFMA, VALU (by kind: transcendental, packed, conversion, other), LDS, vector-memory,
scalar and wait instructions; a quick check of how much non-MFMA issue a loop body carries per MFMA
before paying for a counter run.
"""
from __future__ import annotations

import re
import sys
from collections import Counter


def kernel_lines(path: str, pat: str) -> list[str]:
    out, on = [], False
    for line in open(path):
        if not on and re.match(rf"^_Z\S*{pat}\S*:", line):
            on = True
            continue
        if on:
            if line.startswith(".Lfunc_end"):
                break
            out.append(line.rstrip("\n"))
    return out


def classify(op: str) -> str:
    if op.startswith("v_mfma") or op.startswith("v_smfmac"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "valu_trans"
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith("v_cvt"):
        return "valu_cvt"
    if op.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
        return "valu_lane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_barrier",)):
        return "barrier"
    if op.startswith(("s_nop",)):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, pat)
    labels = {}
    instrs = []  # (line index, opcode)
    for i, ln in enumerate(lines):
        s = ln.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            labels[m.group(1)] = i
            continue
        if not s or s.startswith((";", ".")):
            continue
        instrs.append((i, s.split()[0]))
    total = Counter(classify(op) for _, op in instrs)
    print(f"kernel *{pat}*: {len(instrs)} instructions: " + ", ".join(f"{k} {v}" for k, v in sorted(total.items())))
    for i, ln in enumerate(lines):
        s = ln.strip()
        m = re.match(r"^s_(cbranch_\w+|branch)\s+(\.LBB\S+)", s)
        if not m or m.group(2) not in labels or labels[m.group(2)] >= i:
            continue
        lo = labels[m.group(2)]
        c = Counter(classify(op) for j, op in instrs if lo <= j <= i)
        nm = max(1, c["mfma"])
        valu = c["valu"] + c["valu_trans"] + c["valu_pk"] + c["valu_cvt"] + c["valu_lane"]
        print(f"loop {m.group(2)} (lines {lo}-{i}): mfma {c['mfma']}, valu {valu} ({valu / nm:.2f}/mfma; trans {c['valu_trans']}, "
              f"pk {c['valu_pk']}, cvt {c['valu_cvt']}), lds {c['lds']}, vmem {c['vmem']}, salu {c['salu']}, "
              f"wait {c['wait']}, barrier {c['barrier']}, nop {c['nop']}")


if __name__ == "__main__":
    main()
