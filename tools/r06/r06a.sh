#!/bin/bash
# r06a: optimizer tests, store-hazard pad window / class (verdict r5 item 6), GEMM LDS counters
# (item 1), tile-config comparison on the plain forward shapes.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06a && export TMPDIR=/tmp
O=gpurun_out/r06a
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gpu_train.py -k step_in_backward > $O/train_tests.txt 2>&1; rc=$?
echo "train tests rc=$rc"; [ $rc -le 1 ] || exit $rc
for t in w0 w2 w4 w8 data16 addr16 pk16; do
  FERVIT_LIB=fer-vit_amd/fervit/libfervit_pw_$t.so timeout -k 10 300 $PT tests/test_gpu_kernels.py -k splitk_fold \
    > $O/fold_$t.txt 2>&1; rc=$?
  echo "fold $t rc=$rc $(grep -c PASSED $O/fold_$t.txt) passed $(grep -c FAILED $O/fold_$t.txt) failed"
  [ $rc -le 1 ] || exit $rc
done
for c in fc1 fc2; do
  GEMM_CASE=$c timeout -k 10 150 bash tools/pmc_sq.sh r06a_${c}_a gemm_once.py gemm_8ph > $O/pmc_${c}_a.txt 2>&1 || exit 3
  GEMM_CASE=$c timeout -k 10 150 bash tools/pmc_sq.sh r06a_${c}_b gemm_once.py gemm_8ph SQ_INSTS_LDS SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    > $O/pmc_${c}_b.txt 2>&1 || exit 3
done
echo pmc done
for cfg in 8 5 10; do
  GB_CFG=$cfg GB_ONLY="plain" timeout -k 10 200 python -u tools/gemm_bench.py >> $O/cfg_sweep.txt 2>&1 || exit 4
done
echo sweep done
