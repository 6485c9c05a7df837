#!/bin/bash
# Build the library of a git revision (default HEAD) as fer-vit_amd/fervit/libfervit_base.so, the "base" side of
# an interleaved A/B against the working tree's build (tools/lib_ab.sh).
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/fervit_base_$$
rm -rf $T && mkdir -p $T
git -C "$ROOT" archive "$REV" fer-vit_amd/csrc include | tar -x -C $T
make -C $T/fer-vit_amd/csrc -j8 OUT=$ROOT/fer-vit_amd/fervit/libfervit_base.so $ROOT/fer-vit_amd/fervit/libfervit_base.so > /tmp/build_base.log 2>&1
rm -rf $T
echo "built libfervit_base.so from $REV"
