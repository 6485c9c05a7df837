"""The device build's store-operand padding pass (fer-vit_amd/csrc/store_hazard_pad.py) on small
assembly snippets: an overwrite of a store's data or address register inside the window gets the
missing slots in front of it, on every path through branches; overwrites beyond the window and
writes of other registers are left alone."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("store_hazard_pad",
                                              os.path.join(ROOT, "fer-vit_amd", "csrc", "store_hazard_pad.py"))
shp = importlib.util.module_from_spec(spec)
spec.loader.exec_module(shp)


def run(asm, W=16, cls="all"):
    lines = [l + "\n" for l in asm.strip("\n").split("\n")]
    out, n = shp.pad(lines, W, cls)
    return [l.rstrip("\n") for l in out], n


def nop_slots_before(out, needle):
    i = next(k for k, l in enumerate(out) if needle in l)
    slots = 0
    k = i - 1
    while k >= 0 and "store operand hazard pad" in out[k]:
        slots += int(out[k].split()[1]) + 1
        k -= 1
    return slots


def test_data_overwrite_padded_to_window():
    out, n = run("""
\tbuffer_store_dwordx4 v[156:159], v195, s[8:11], s12 offen
\ts_lshl_b32 s70, s34, 6
\ts_lshl_b32 s71, s34, 7
\tv_pk_mul_f32 v[156:157], v[192:193], v[154:155] op_sel_hi:[0,1]
""")
    assert n == 1
    assert nop_slots_before(out, "v_pk_mul_f32") == 16 - 2  # two SALU slots already there


def test_default_tracks_data_operands_in_a_4_slot_window():
    """The shipped setting (measured class and window: profiles/r06a_store_pad_window.txt): a store's data
    registers 4 slots, its address registers not at all."""
    lines = [l + "\n" for l in """
\tbuffer_store_dwordx4 v[156:159], v195, s[8:11], s12 offen
\ts_lshl_b32 s70, s34, 6
\tv_pk_mul_f32 v[156:157], v[192:193], v[154:155] op_sel_hi:[0,1]
\tglobal_store_dwordx4 v[38:39], v[0:3], off
\tv_lshl_add_u64 v[38:39], v[38:39], 0, s[4:5]
""".strip("\n").split("\n")]
    assert shp.W_DEFAULT == 4 and shp.CLASS_DEFAULT == "data"
    out, n = shp.pad(lines, shp.W_DEFAULT)
    out = [l.rstrip("\n") for l in out]
    assert n == 1
    assert nop_slots_before(out, "v_pk_mul_f32") == 3
    assert nop_slots_before(out, "v_lshl_add_u64") == 0


def test_address_overwrite_padded():
    out, n = run("""
\tglobal_store_dwordx4 v[38:39], v[0:3], off
\ts_or_b64 exec, exec, s[14:15]
\tv_lshl_add_u64 v[38:39], v[38:39], 0, s[4:5]
""")
    assert n == 1 and nop_slots_before(out, "v_lshl_add_u64") == 15


def test_agpr_data_and_lds_read_tracked():
    out, n = run("""
\tglobal_store_dwordx4 v[8:9], a[0:3], off
\tv_accvgpr_write_b32 a1, v5
\tbuffer_store_dwordx4 v[4:7], v1, s[8:11], 0 offen
\tds_read_b128 v[4:7], v2
""")
    assert n == 2


def test_unrelated_and_far_writes_untouched():
    far = "\n".join(["\tv_add_u32_e32 v10, 1, v10"] * 16)
    out, n = run(f"""
\tbuffer_store_dwordx4 v[0:3], v4, s[8:11], 0 offen
\tv_mov_b32_e32 v5, 0
{far}
\tv_mov_b32_e32 v0, 0
""")
    assert n == 0


def test_branch_targets_followed():
    out, n = run("""
\tbuffer_store_dwordx4 v[0:3], v4, s[8:11], 0 offen
\ts_cbranch_execz .LBB0_2
\tv_mov_b32_e32 v9, 0
\ts_branch .LBB0_3
.LBB0_2:
\tv_mov_b32_e32 v1, 0
.LBB0_3:
\tv_mov_b32_e32 v2, 0
""")
    # the taken path reaches v1 one slot (the branch) after the store; the fallthrough reaches v2 after three
    assert nop_slots_before(out, "v_mov_b32_e32 v1, 0") == 15
    assert nop_slots_before(out, "v_mov_b32_e32 v2, 0") == 13
    assert n == 2


def test_inline_asm_sgpr_read_after_valu_write_padded():
    # the round-4 / round-5 fault: a spilled SGPR reloaded by v_readlane right before the inline-asm
    # claim atomic that takes the pair as its address
    lines = [l + "\n" for l in """
\tv_readlane_b32 s6, v255, 3
\tv_mov_b32_e32 v0, 1
\tv_readlane_b32 s7, v255, 4
\t;;#ASMSTART
\tglobal_atomic_add v243, v194, v0, s[6:7] sc0
\t;;#ASMEND
\ts_mov_b32 s8, s9
\t;;#ASMSTART
\tglobal_atomic_add v243, v194, v0, s[8:9] sc0
\t;;#ASMEND
""".strip("\n").split("\n")]
    out, n = shp.pad_asm_sgpr(lines)
    out = [l.rstrip("\n") for l in out]
    assert n == 1
    i = next(k for k, l in enumerate(out) if "s[6:7]" in l)
    assert out[i - 1].strip().startswith("s_nop 4")  # the full 5 wait states in front of the atomic
    # an SGPR written by SALU needs no pad
    j = next(k for k, l in enumerate(out) if "s[8:9]" in l)
    assert "s_nop" not in out[j - 1]


def test_inline_asm_sgpr_pad_counts_wait_states_and_labels():
    lines = [l + "\n" for l in """
\tv_readfirstlane_b32 s5, v1
\ts_nop 1
\tv_mov_b32_e32 v2, 0
\t;;#ASMSTART
\tbuffer_load_dwordx4 v3, s[8:11], s5 offen lds
\t;;#ASMEND
.LBB0_1:
\t;;#ASMSTART
\tbuffer_load_dwordx4 v3, s[8:11], 0 offen lds
\t;;#ASMEND
""".strip("\n").split("\n")]
    out, n = shp.pad_asm_sgpr(lines)
    out = [l.rstrip("\n") for l in out]
    assert n == 2
    i = next(k for k, l in enumerate(out) if "s5 offen" in l)
    assert out[i - 1].strip().startswith("s_nop 1")  # 3 slots there (s_nop 1 + v_mov): 2 more
    j = next(k for k, l in enumerate(out) if ", 0 offen lds" in l)
    assert out[j - 1].strip().startswith("s_nop 4")  # a label right before: assume the worst


def test_built_assembly_has_no_inline_asm_sgpr_hazard():
    """The assembly the library is built from (csrc/build/*.pad.s, present after build()) has no
    inline-asm vector-memory instruction reading a VALU-written SGPR within 5 wait states."""
    import glob

    import pytest

    files = glob.glob(os.path.join(ROOT, "fer-vit_amd", "csrc", "build", "*.pad.s"))
    if not files:
        pytest.skip("library not built in this tree")
    spec2 = importlib.util.spec_from_file_location("check_asm_sgpr_hazard",
                                                   os.path.join(ROOT, "tools", "check_asm_sgpr_hazard.py"))
    chk = importlib.util.module_from_spec(spec2)
    spec2.loader.exec_module(chk)
    for f in files:
        assert chk.scan(f) == [], f


def test_lds_returning_ops_tracked():
    # a ds_bpermute writing a store's data register right after the store is padded like an LDS read
    out, n = run("""
\tbuffer_store_dword v5, v1, s[8:11], 0 offen
\tds_bpermute_b32 v5, v2, v3
\tbuffer_store_dword v6, v1, s[8:11], 0 offen
\tds_write_b32 v6, v7
""")
    assert n == 1 and nop_slots_before(out, "ds_bpermute_b32") == 16


def test_atomic_operands_tracked():
    out, n = run("""
\tglobal_atomic_add v235, v2, v3, s[56:57] sc0
\tv_mov_b32_e32 v3, 0
""")
    assert n == 1 and nop_slots_before(out, "v_mov_b32_e32 v3, 0") == 16
