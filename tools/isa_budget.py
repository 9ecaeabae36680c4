#!/usr/bin/env python3
"""Instruction budget of a kernel's loops, read off the compiler's ISA
(hipcc --cuda-device-only -S): per basic block, the wave instructions by
class (VALU, SALU, LDS, VMEM, SMEM, branch, waitcnt) and the block's loop
nesting from the compiler's annotations.

usage: isa_budget.py FILE.s KERNEL_SUBSTRING [BLOCK ...]
  with BLOCK labels (e.g. .LBB1_61 .LBB1_63 .LBB1_65 .LBB1_60) also prints
  the sum over those blocks: one path through a loop body.
"""
import re
import sys

CLASSES = ("valu", "salu", "lds", "vmem", "smem", "branch", "wait", "other")


def klass(op):
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
        return "branch"
    if op.startswith(("ds_", "buffer_load_lds")):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_memtime")):
        return "smem"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def blocks(path, kernel):
    """[(label, depth note, {class: count})] of the first function whose
    name contains `kernel`"""
    out, cur, inside = [], None, False
    for line in open(path):
        s = line.rstrip("\n")
        if not inside:
            if re.match(r"^_Z\w*:", s) and kernel in s.split(":")[0]:
                inside = True
                cur = ["entry", "", dict.fromkeys(CLASSES, 0)]
                out.append(cur)
            continue
        if re.match(r"^_Z\w*:", s) or s.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):\s*(;.*)?$", s)
        if m:
            note = (m.group(2) or "").lstrip("; ").strip()
            cur = [m.group(1).replace("; ", ""), note, dict.fromkeys(CLASSES, 0)]
            out.append(cur)
            continue
        t = s.strip()
        if not t or t.startswith((";", ".", "//")):
            continue
        cur[2][klass(t.split()[0])] += 1
    return out


def main():
    if len(sys.argv) < 3:
        sys.exit(__doc__)
    path, kernel, picks = sys.argv[1], sys.argv[2], sys.argv[3:]
    bl = blocks(path, kernel)
    print("%-10s %s  %s" % ("block", " ".join("%6s" % c for c in CLASSES), "loop"))
    for lab, note, c in bl:
        print("%-10s %s  %s" % (lab, " ".join("%6d" % c[k] for k in CLASSES), note[:60]))
    if picks:
        tot = dict.fromkeys(CLASSES, 0)
        for lab, _, c in bl:
            if lab in picks:
                for k in CLASSES:
                    tot[k] += c[k]
        print("%-10s %s  %s" % ("PATH", " ".join("%6d" % tot[k] for k in CLASSES), "+".join(picks)))


if __name__ == "__main__":
    main()
