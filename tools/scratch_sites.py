"""Scratch (spill) accesses of one kernel of the built library, per basic block, with the block's size.

    python tools/scratch_sites.py <kernel-substring>
"""
import collections
import re
import sys

import isa_count as ic


def main():
    t = ic.disassemble(sys.argv[2] if len(sys.argv) > 2 else
                       __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "of_dis_amd",
                                                  "csrc", "build", "ofdis_kernels.o"))
    name, body = ic.parse_kernel(t, sys.argv[1])
    lines = [l.strip().split("//")[0].strip() for l in body.splitlines()[1:]]
    lines = [l for l in lines if l and not l.startswith(";")]
    lab, size, cnt = None, collections.Counter(), collections.Counter()
    for l in lines:
        m = re.match(r"^[0-9a-f]+ <(L\d+)>:", l)
        if m:
            lab = m.group(1)
            continue
        size[lab] += 1
        if l.startswith("scratch_"):
            cnt[(lab, l.split()[0])] += 1
    print(name)
    for (b, op), v in sorted(cnt.items()):
        print(f"  {b} (block of {size[b]}): {op} x{v}")


if __name__ == "__main__":
    main()
