"""Static check of the device assembly: an inline-asm vector-memory instruction (between ;;#ASMSTART and
;;#ASMEND, where LLVM's hazard recognizer does not look) that reads an SGPR a VALU instruction
(v_readlane / v_readfirstlane / v_cmp / v_*_co ... with an SGPR destination) wrote fewer than 5 wait
states earlier. gfx9 / CDNA: "VALU writes SGPR -> VMEM reads that SGPR" needs 5 wait states; with
fewer, the memory instruction can read the SGPR's OLD value, e.g. a stale 64-bit address.

    python tools/check_asm_sgpr_hazard.py file.s [function-substring]
    python tools/check_asm_sgpr_hazard.py --dis file.dis [function-substring]
(--dis: an llvm-objdump -d listing of a code object, which has no inline-asm markers: every
vector-memory instruction is checked, so compiler-scheduled ones show up only if the compiler
missed the hazard too.)
"""
import re
import sys

SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
VMEM = re.compile(r"^\s*(global|buffer|flat|scratch)_\w+")


def sregs(text):
    out = set()
    for m in SREG.finditer(text):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def valu_sdst(t):
    if not t.startswith("v_"):
        return set()
    parts = t.split(None, 1)
    if len(parts) < 2:
        return set()
    return sregs(parts[1].split(",")[0])


def nslots(t):
    m = re.match(r"s_nop\s+(\d+)", t)
    return int(m.group(1)) + 1 if m else 1


def scan(path, filt="", dis=False):
    lines = open(path).readlines()
    if dis:  # "<sym>:" headers, instructions with "// addr: encoding" comments
        lines = [re.sub(r"^[0-9a-f]+ <(\S+)>:", r"\1:", l).split("//")[0] + "\n" for l in lines]
    fn, inasm, hits = "?", dis, []
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\w+):", l)
        if m:
            fn = m.group(1)
        t = l.strip()
        if t.startswith(";;#ASMSTART"):
            inasm = True
            continue
        if t.startswith(";;#ASMEND"):
            inasm = False
            continue
        if not inasm or filt not in fn or not VMEM.match(t):
            continue
        need = sregs(t.split(None, 1)[1]) if len(t.split(None, 1)) > 1 else set()
        used, j = 0, i - 1
        while j >= 0 and used < 5:
            tt = lines[j].strip()
            if not tt or tt.startswith((";", ".")) or tt.endswith(":"):
                j -= 1
                continue
            if valu_sdst(tt) & need:
                hits.append((fn, i + 1, used, tt, t))
                break
            used += nslots(tt)
            j -= 1
    return hits


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--dis"]
    hits = scan(args[0], args[1] if len(args) > 1 else "", dis="--dis" in sys.argv)
    for fn, ln, used, w, t in hits:
        print(f"{fn[:70]} line {ln}: {used} wait states: {w[:50]}  ->  {t[:60]}")
    print(f"{len(hits)} {'VMEM' if '--dis' in sys.argv else 'inline-asm VMEM'} instructions read a VALU-written SGPR within 5 wait states")
