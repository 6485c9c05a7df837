"""CPU checks of the C ABI: the built library loads and exports every symbol that
include/fervit.h declares (no compute calls — there is no GPU here), and the ctypes
signature table covers exactly that set."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "fervit.h")
LIB = os.path.join(ROOT, "fer-vit_amd", "fervit", "libfervit.so")


def declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fer_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    for n in ("fer_gemm", "fer_layernorm_fwd", "fer_layernorm_bwd", "fer_attention_fwd", "fer_attention_bwd",
              "fer_adamw", "fer_cross_entropy", "fer_wplus_fwd", "fer_decompose", "fer_last_error"):
        assert n in names


@pytest.mark.skipif(not os.path.exists(LIB), reason="libfervit.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.fer_version and ctypes.cast(lib.fer_last_error, ctypes.c_void_p).value


@pytest.mark.skipif(not os.path.exists(LIB), reason="libfervit.so not built")
def test_ctypes_table_matches_header():
    from fervit._lib import SIGNATURES, lib

    L = lib()
    assert set(SIGNATURES) == set(declared())
    assert L.fer_version().decode().startswith("fervit")
