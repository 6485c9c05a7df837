"""Build step: pad gfx950 device assembly so that no VALU instruction (or data-returning LDS instruction)
overwrites a VGPR / AGPR holding the DATA of a preceding vector-memory store or atomic within W issue
slots (default W = 4).

Why: on MI355X the hardware read of a store's data registers can trail its issue by more than the wait
states the compiler accounts for. Measured (DESIGN.md sections 10-11, profiles/r05_store_war_*,
profiles/r06a_store_pad_window.txt): the in-launch split-K fold's buffer_store_dwordx4, followed within two
slots by VALU writes of its data registers (v_pk_mul_f32 among others), stored the new value of one dword
in 4 lanes of 16 on every launch. One library per pass setting, each running that reproducer once
(round 6): no pads -> wrong values; every operand (data and address) at W = 2, 4, 8 -> exact; data
operands only at W = 2, 4, 16 -> exact; address operands only at W = 16 -> wrong; v_pk_* writers only at
W = 16 -> wrong. So the class is "a VALU / LDS-read write of a store's DATA registers" (any opcode), and a
2-slot window suffices on that reproducer; the default keeps twice that. (The 128^2 epilogue's
"address-register" case of round 5 was the LDS race its barrier fixed: profiles/r05p_gemm128_stress_after_fix.txt,
0 of 149 with no pads at all.) PAD_W / PAD_CLASS (data | addr | all) / PAD_WRITER (an opcode prefix) select
other settings for experiment builds.
The pass walks each store's following instructions in program order; when a VALU (v_*) or an LDS read writes one of
the tracked registers less than W slots after it, an s_nop of the missing slots goes in front of that
instruction, on every path: branches are followed into their targets (both successors of a conditional
branch). Every other instruction is left as it is.

The same pass also pads inline assembly against "VALU writes SGPR -> VMEM reads that SGPR" (5 wait
states on gfx9 / CDNA): LLVM's hazard recognizer does not look at inline-asm operands, and a
v_readlane_b32 reloading a spilled SGPR right before the work-queue claim (an inline-asm
global_atomic_add whose 64-bit address is an SGPR pair) let the atomic read the pair's old value:
the round-4 / round-5 GPU faults of the pipelined GEMM schedule (DESIGN.md section 10,
profiles/r05w_*, tools/check_asm_sgpr_hazard.py). Every inline-asm vector-memory instruction that
reads an SGPR gets an s_nop in front of it when a VALU instruction writing that SGPR is fewer than 5
wait states before it, or when a label (another block's path) comes first.

    python store_hazard_pad.py in.s out.s [W]
"""
import os
import re
import sys

W_DEFAULT = 4
CLASS_DEFAULT = "data"

# vector-memory stores and atomics (an atomic reads its address and data registers the same way)
STORE = re.compile(r"^\s*((global|buffer|flat|scratch)_store_\w+|(global|buffer|flat)_atomic_\w+)")
BRANCH = re.compile(r"^\s*s_(branch|cbranch_\w+|setpc_b64|swappc_b64|endpgm\w*)\b")
LABEL = re.compile(r"^[.\w$]+:")
REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            out.update((m.group(3), r) for r in range(int(m.group(4)), int(m.group(5)) + 1))
    return out


def data_index(op, mods):
    """Operand position of a store's / atomic's data: buffer_* puts vdata first; global_ / flat_ / scratch_
    stores put the address first (vaddr, vdata, ...); a returning global / flat atomic (sc0) has vdst,
    vaddr, vdata."""
    if op.startswith("buffer_"):
        return 0
    if "_atomic" in op and re.search(r"\bsc0\b", mods):
        return 2
    return 1


def store_regs(line, cls="all"):
    """Registers a store reads: every v/a register among its operands (data and address). cls: "data" =
    only the data operand, "addr" = only the rest."""
    parts = line.split(None, 1)
    body = parts[1] if len(parts) > 1 else ""
    body = body.split("//")[0].split(";")[0]
    if cls == "all":
        return regs(body)
    ops = [o.strip() for o in body.split(",")]
    di = data_index(parts[0].strip(), body)
    data = regs(ops[di].split()[0]) if len(ops) > di and ops[di] else set()
    return data if cls == "data" else regs(body) - data


LDS_RET = re.compile(r"^ds_(read|load|bpermute|permute|swizzle)|^ds_\w*_rtn")


WRITER = os.environ.get("PAD_WRITER", "")  # experiment builds only: pad only writers with this prefix


def valu_dst(line):
    """Registers written soon after issue: VALU destinations and the destinations of LDS instructions
    that return data (reads, ds_bpermute / ds_permute / ds_swizzle, returning atomics: tens of cycles);
    vector-memory loads return far later and are not tracked."""
    t = line.strip()
    if not (t.startswith("v_") or LDS_RET.match(t)):
        return set()
    if WRITER and not t.startswith(WRITER):
        return set()
    parts = t.split(None, 1)
    if len(parts) < 2:
        return set()
    first = parts[1].split(",")[0].strip()
    return regs(first)


def slots(line):
    t = line.strip()
    m = re.match(r"s_nop\s+(\d+)", t)
    if m:
        return int(m.group(1)) + 1
    return 1


def is_instr(line):
    t = line.strip()
    return bool(t) and not t.startswith((".", ";", "//")) and not LABEL.match(t)


def nops(n, indent="\t"):
    out = []
    while n > 0:
        k = min(n, 8)
        out.append(f"{indent}s_nop {k - 1}\t; store operand hazard pad\n")
        n -= k
    return out


def pad(lines, W, cls=CLASS_DEFAULT):
    """Pads in front of every VALU / LDS-read write of a store's register on any path that reaches it
    less than W slots after the store: branches are followed into their targets (both ways for a
    conditional one), so a window that leaves a block is padded only where an overwrite happens."""
    labels = {}
    for i, l in enumerate(lines):
        m = LABEL.match(l.strip())
        if m:
            labels[l.strip()[:-1]] = i
    insert_before = {}  # line index -> slots to pad in front of it

    def walk(j, used, live, seen):
        while j < len(lines) and used < W:
            t = lines[j]
            s_ = t.strip()
            if not is_instr(t):
                j += 1
                continue
            if valu_dst(t) & live:
                insert_before[j] = max(insert_before.get(j, 0), W - used)
                return
            if BRANCH.match(t):
                op = s_.split()[0]
                if op.startswith("s_endpgm") or op.startswith(("s_setpc", "s_swappc")):
                    return
                target = s_.split()[1] if len(s_.split()) > 1 else None
                used += slots(t)
                if target in labels and (target, used) not in seen:
                    seen.add((target, used))
                    walk(labels[target] + 1, used, live, seen)
                if op == "s_branch":
                    return
                j += 1
                continue
            used += slots(t)
            j += 1

    for i, l in enumerate(lines):
        if not STORE.match(l):
            continue
        live = store_regs(l, cls)
        if live:
            walk(i + 1, 0, live, set())
    out = []
    for i, l in enumerate(lines):
        if i in insert_before:
            out.extend(nops(insert_before[i]))
        out.append(l)
    return out, len(insert_before)


VMEM = re.compile(r"^\s*(global|buffer|flat|scratch)_\w+")
SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
SGPR_WS = 5  # VALU writes SGPR -> VMEM reads that SGPR


def sregs(text):
    out = set()
    for m in SREG.finditer(text):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def valu_sdst(line):
    t = line.strip()
    if not t.startswith("v_"):
        return set()
    parts = t.split(None, 1)
    return sregs(parts[1].split(",")[0]) if len(parts) > 1 else set()


def pad_asm_sgpr(lines):
    """s_nop in front of every inline-asm VMEM instruction that reads an SGPR written by a VALU
    instruction fewer than SGPR_WS wait states earlier (or with a label within that window)."""
    out, n, inasm = [], 0, False
    for i, l in enumerate(lines):
        t = l.strip()
        if t.startswith(";;#ASMSTART"):
            inasm = True
        elif t.startswith(";;#ASMEND"):
            inasm = False
        elif inasm and VMEM.match(l):
            need = sregs(t.split(None, 1)[1]) if len(t.split(None, 1)) > 1 else set()
            used, j, short = 0, i - 1, 0
            while need and j >= 0 and used < SGPR_WS:
                tj = lines[j].strip()
                if LABEL.match(tj):
                    short = SGPR_WS - used  # another path may reach here: assume the worst
                    break
                if is_instr(lines[j]):
                    if valu_sdst(lines[j]) & need:
                        short = SGPR_WS - used
                        break
                    used += slots(lines[j])
                j -= 1
            if short > 0:
                out.append(f"\ts_nop {short - 1}\t; inline-asm SGPR read hazard pad\n")
                n += 1
        out.append(l)
    return out, n


def main():
    src, dst = sys.argv[1], sys.argv[2]
    W = int(sys.argv[3]) if len(sys.argv) > 3 else W_DEFAULT
    with open(src) as f:
        lines = f.readlines()
    out, n = pad(lines, W, os.environ.get("PAD_CLASS", CLASS_DEFAULT))
    na = 0
    if os.environ.get("PAD_SGPR", "1") != "0":  # (PAD_SGPR=0: A/B builds only)
        out, na = pad_asm_sgpr(out)
    with open(dst, "w") as f:
        f.writelines(out)
    print(f"store_hazard_pad: {n} pads ({W} slots, {os.environ.get('PAD_CLASS', CLASS_DEFAULT)} operands), "
          f"{na} inline-asm SGPR pads in {src}", file=sys.stderr)


if __name__ == "__main__":
    main()
