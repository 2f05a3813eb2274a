"""Instruction mix of the MFMA loop(s) of one kernel in a gfx950 ISA dump
(hipcc --cuda-device-only -S).  A loop = a label whose block range ends in a
branch back to it; reports per-loop counts of MFMA / VALU / LDS / SALU / s_nop /
waitcnt, used for the issue models in bench.py and DESIGN.md.

usage: python tools/isa_loop_mix.py featnn.s 'featnn_row8ILi2ELi8ELb1E'"""
import re
import sys
from collections import Counter


def kernel_lines(path, key):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + key + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    return lines[start:end + 1]


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op == "s_nop":
        return "s_nop"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    body = kernel_lines(sys.argv[1], sys.argv[2])
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_cbranch_\w+\s+(\.LBB\S+)|^\s+s_branch\s+(\.LBB\S+)", l)
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        j = labels.get(tgt)
        if j is None or j >= i:
            continue
        c = Counter()
        ops = Counter()
        for l2 in body[j:i + 1]:
            t = l2.strip().split()
            if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
                continue
            c[classify(t[0])] += 1
            if classify(t[0]) == "valu":
                ops[t[0]] += 1
        if c["mfma"] or "--all" in sys.argv:
            print(f"loop {tgt} lines {j}-{i}: {dict(c)}")
            print("   valu:", ", ".join(f"{k} {v}" for k, v in ops.most_common(12)))


if __name__ == "__main__":
    main()
