#!/bin/bash
# verdict r5 item 6, second pass: the data-operand class at windows 2 and 4
set -e
cd "$(dirname "$0")/../fer-vit_amd/csrc"
for w in 2 4; do
  PAD_CLASS=data make -j8 BUILD=build_pw_data$w OUT=../fervit/libfervit_pw_data$w.so PAD_W=$w ../fervit/libfervit_pw_data$w.so \
    > /tmp/pw_data$w.log 2>&1
  grep 'store_hazard_pad' /tmp/pw_data$w.log | grep gemm
done
