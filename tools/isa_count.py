"""Instruction counts of one kernel of the built library, per basic-block region.

    python tools/isa_count.py <kernel-substring> [--obj of_dis_amd/csrc/build/ofdis_kernels.o] [--blocks]

Extracts the gfx950 code object from the object file's .hip_fatbin section, disassembles it and prints, for
the first kernel whose demangled name contains the substring: the total instruction count by class and,
for every backward branch (a loop), the classes of the instructions between its target and itself.
With --blocks every basic block (label) is listed with its class counts.  Static counts: a loop body's
count is its per-trip issue count when it has no inner branches.
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disassemble(obj):
    tmp = tempfile.mkdtemp(prefix="isa_")
    fat, co = os.path.join(tmp, "fat.bin"), os.path.join(tmp, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "--symbolize-operands", co],
                         check=True, capture_output=True, text=True).stdout
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
    return r.stdout.splitlines()


def klass(op):
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith(("v_mfma", "v_smfmac")):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer", "s_store", "s_memtime", "s_dcache")):
        return "smem"
    if op.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_sleep", "s_setprio")):
        return "sync"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


def parse_kernel(text, pattern):
    heads = [(m.start(), m.group(1)) for m in re.finditer(r"^[0-9a-f]+ <([^>L][^>]*)>:", text, re.M)]
    names = demangle([h[1] for h in heads])
    for i, (pos, _) in enumerate(heads):
        if pattern in names[i]:
            end = heads[i + 1][0] if i + 1 < len(heads) else len(text)
            return names[i], text[pos:end]
    sys.exit(f"no kernel matches {pattern!r}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pattern")
    ap.add_argument("--obj", default=os.path.join(os.path.dirname(__file__), "..", "of_dis_amd", "csrc", "build",
                                                  "ofdis_kernels.o"))
    ap.add_argument("--blocks", action="store_true")
    args = ap.parse_args()
    name, body = parse_kernel(disassemble(args.obj), args.pattern)
    insts = []  # (label or None, opcode, text)
    label = None
    for line in body.splitlines()[1:]:
        m = re.match(r"^[0-9a-f]+ <(L\d+)>:", line.strip())
        if m:
            label = m.group(1)
            continue
        s = line.strip()
        if not s or s.startswith(";"):
            continue
        s = s.split("//")[0].strip()
        op = s.split()[0]
        insts.append((label, op, s))
        label = None
    print(name)
    tot = collections.Counter(klass(op) for _, op, _ in insts)
    print("total", len(insts), dict(tot))
    pos = {}
    for i, (lab, _, _) in enumerate(insts):
        if lab:
            pos[lab] = i
    for i, (_, op, s) in enumerate(insts):
        if op in ("s_cbranch_scc0", "s_cbranch_scc1", "s_cbranch_vccz", "s_cbranch_vccnz", "s_cbranch_execz",
                  "s_cbranch_execnz", "s_branch"):
            m = re.search(r"\b(L\d+)\b", s)
            if m and m.group(1) in pos and pos[m.group(1)] <= i:
                j = pos[m.group(1)]
                c = collections.Counter(klass(o) for _, o, _ in insts[j:i + 1])
                print(f"loop {m.group(1)} [{j}..{i}] {i - j + 1} insts", dict(c))
    if args.blocks:
        cur, start = None, 0
        for i, (lab, _, _) in enumerate(insts + [("END", "", "")]):
            if lab:
                if cur is not None:
                    c = collections.Counter(klass(o) for _, o, _ in insts[start:i])
                    print(f"  block {cur} [{start}..{i - 1}] {i - start}", dict(c))
                cur, start = lab, i


if __name__ == "__main__":
    main()
