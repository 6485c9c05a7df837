#!/bin/bash
# Verdict r5 item 6: libraries whose store-operand pad pass uses a smaller window or only one operand
# class, each to run test_wgrad_splitk_fold_bit_exact (the fold reproducer: deterministic wrong values
# when the hazard is not padded) once: FERVIT_LIB=fer-vit_amd/fervit/libfervit_pw_<tag>.so.
set -e
cd "$(dirname "$0")/../fer-vit_amd/csrc"
build() {  # tag W [env...]
  local tag=$1 w=$2; shift 2
  env "$@" make -j8 BUILD=build_pw_$tag OUT=../fervit/libfervit_pw_$tag.so PAD_W=$w ../fervit/libfervit_pw_$tag.so \
    > /tmp/pw_$tag.log 2>&1
  grep 'store_hazard_pad' /tmp/pw_$tag.log | grep gemm
}
build w0 0
build w2 2
build w4 4
build w8 8
build data16 16 PAD_CLASS=data
build addr16 16 PAD_CLASS=addr
build pk16 16 PAD_WRITER=v_pk_
