"""Static scan for a write-after-read hazard on gfx950 store data: a VALU instruction that writes a
VGPR read as data by a preceding 16-byte (dwordx4) vector-memory store within a few instructions.
Measured (profiles/r05_fold_store_war.txt): with two SALU instructions between a
buffer_store_dwordx4 and a v_pk_mul_f32 overwriting its data registers, the store wrote the new
value of one dword in 4 lanes of every 16 -- the compiler's wait-state count for this hazard is
not enough on this hardware.

    python tools/check_store_war.py [window] [files...]

Compiles the listed csrc files (default: every .hip) to gfx950 assembly and reports, per kernel,
each dwordx4 store followed within `window` instructions (default 4) by a VALU write to one of its
data VGPRs, with the instructions in between."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fer-vit_amd", "csrc")


def regs(tok):
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def scan(asm, window):
    lines = [l.strip() for l in asm.split("\n")]
    hits, kern = [], None
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            kern = m.group(1)
        if not re.match(r"(buffer|global|flat|scratch)_store_dwordx4\b", l):
            continue
        ops = [o.strip() for o in l.split(None, 1)[1].split(",")]
        data = regs(ops[1] if l.startswith("global") or l.startswith("flat") or l.startswith("scratch") else ops[0])
        seen, between = 0, []
        for j in range(i + 1, len(lines)):
            t = lines[j]
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            if t.startswith(("s_endpgm", "s_branch", "s_cbranch", "s_setpc")):
                break
            seen += 1
            if seen > window:
                break
            if t.startswith("v_"):
                dst = t.split(None, 1)[1].split(",")[0].strip() if " " in t else ""
                if regs(dst) & data:
                    hits.append((kern, i + 1, l, between[:], t))
                    break
            between.append(t.split()[0])
    return hits


def main():
    window = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    files = sys.argv[2:] or sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    total = 0
    with tempfile.TemporaryDirectory() as td:
        for f in files:
            out = os.path.join(td, f + ".s")
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                            "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S", "-x", "hip",
                            os.path.join(CSRC, f), "-o", out], check=True, stderr=subprocess.DEVNULL)
            hits = scan(open(out).read(), window)
            total += len(hits)
            kerns = {}
            for k, *_ in hits:
                kerns[k] = kerns.get(k, 0) + 1
            print(f"{f}: {len(hits)} store-data overwrites within {window} instructions in {len(kerns)} kernels")
            for k, n in sorted(kerns.items(), key=lambda kv: -kv[1])[:40]:
                ex = next(h for h in hits if h[0] == k)
                print(f"  {n:4d}  {k[:100]}\n        e.g. line {ex[1]}: {ex[2]}  -> {ex[4]}  (between: {' '.join(ex[3])})")
    print("total", total)


if __name__ == "__main__":
    main()
