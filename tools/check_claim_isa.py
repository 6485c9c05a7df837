"""Static check of the inline-asm work-queue claims: `wq_claim_issue` and the 8-phase
GEMM's claim are `global_atomic_add ... sc0` written as inline asm, so the compiler does not know the
destination VGPR is still pending. A copy, spill or overwrite of that register before the explicit
`s_waitcnt vmcnt(0)` would read or clobber it before the atomic returns.

    python tools/check_claim_isa.py [out.txt]

Compiles gemm.hip and attention.hip to gfx950 assembly (hipcc -S, device only) and, for every
inline-asm returning atomic, walks the instructions that follow it in program order up to the first
`s_waitcnt` that waits for vmcnt(0) (or the kernel's end) and reports any instruction that reads or
writes the destination register (spills included: a spill is a read). Instructions on a branch
that cannot run after the atomic (the other arm of the `wq.q` test) show up too; each such hit is
listed with its basic block so it can be checked by hand.
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fer-vit_amd", "csrc")


def regs_of(tok):
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def scan(asm):
    lines = asm.split("\n")
    out = []
    kern, block, in_asm = None, None, False
    for i, l in enumerate(lines):
        s = l.strip()
        m = re.match(r"^(_Z\S+):", l)
        if m:
            kern = m.group(1)
        if re.match(r"^\.LBB\S+:|^; %bb", s):
            block = s.split()[0]
        if s == ";;#ASMSTART":
            in_asm = True
        elif s == ";;#ASMEND":
            in_asm = False
        if not (in_asm and s.startswith("global_atomic") and " sc0" in s):
            continue
        dst = s.split()[1].rstrip(",")
        dregs = regs_of(dst)
        hits, end = [], None
        blk = block
        for j in range(i + 1, len(lines)):
            t = lines[j].strip()
            if re.match(r"^\.LBB\S+:|^; %bb", t):
                blk = t.split()[0]
            if re.match(r"^(_Z\S+):", lines[j]) or t.startswith("s_endpgm") or t.startswith(".Lfunc_end"):
                end = f"end of kernel at line {j + 1}"
                break
            if t.startswith("s_waitcnt") and "vmcnt(0)" in t:
                end = f"s_waitcnt vmcnt(0) at line {j + 1}"
                break
            if not t or t.startswith((";", ".")):
                continue
            ops = [o.strip() for o in t.split(None, 1)[1].split(",")] if " " in t else []
            used = set()
            for o in ops:
                used |= regs_of(o.split()[0]) if o else set()
            if used & dregs:
                hits.append(f"    line {j + 1} [{blk}]: {t}")
        out.append((kern, i + 1, s, end, hits))
    return out


def main():
    dest = sys.argv[1] if len(sys.argv) > 1 else None
    report = []
    with tempfile.TemporaryDirectory() as td:
        for src in ("gemm.hip", "attention.hip"):
            asm_path = os.path.join(td, src + ".s")
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                            "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S", "-x", "hip",
                            os.path.join(CSRC, src), "-o", asm_path], check=True, stderr=subprocess.DEVNULL)
            for kern, ln, ins, end, hits in scan(open(asm_path).read()):
                report.append(f"{src}:{ln} {kern[:90]}\n  {ins}\n  until {end}: "
                              + (f"{len(hits)} access(es) to the destination" if hits else "destination untouched"))
                report.extend(hits)
    text = "\n".join(report) + "\n"
    print(text)
    if dest:
        with open(dest, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
