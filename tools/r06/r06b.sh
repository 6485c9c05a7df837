#!/bin/bash
# r06b: ring ping-pong main loop (bit-exactness test, A/B vs the 8-phase loop alone), data-class pad windows 2 / 4
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06b && export TMPDIR=/tmp
O=gpurun_out/r06b
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_gpu_kernels.py -k "main_loop_ring or 8phase_epilogue_kinds or persistent_many" > $O/loop_tests.txt 2>&1; rc=$?
echo "loop tests rc=$rc $(grep -c PASSED $O/loop_tests.txt) passed $(grep -c FAILED $O/loop_tests.txt) failed"; [ $rc -le 1 ] || exit $rc
GB_LOOP=ab timeout -k 10 400 python -u tools/gemm_bench.py > $O/loop_ab.txt 2>&1 || exit 4
echo "bench done"
for t in data2 data4; do
  FERVIT_LIB=fer-vit_amd/fervit/libfervit_pw_$t.so timeout -k 10 300 $PT tests/test_gpu_kernels.py -k splitk_fold \
    > $O/fold_$t.txt 2>&1; rc=$?
  echo "fold $t rc=$rc $(grep -c PASSED $O/fold_$t.txt) passed"
  [ $rc -le 1 ] || exit $rc
done
