#!/bin/bash
# r06c: five-stage ring ping-pong (DMA-latency hypothesis), pp kernel (cfg 10) on the fused epilogue shapes
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06c && export TMPDIR=/tmp
O=gpurun_out/r06c
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_gpu_kernels.py -k "main_loop_ring" > $O/loop_tests.txt 2>&1; rc=$?
echo "loop tests rc=$rc $(grep -c PASSED $O/loop_tests.txt) passed $(grep -c FAILED $O/loop_tests.txt) failed"; [ $rc -eq 0 ] || exit $rc
GB_LOOP=ab GB_ONLY=fwd timeout -k 10 400 python -u tools/gemm_bench.py > $O/loop_ab.txt 2>&1 || exit 4
echo "bench done"
GB_CFG=10 timeout -k 10 400 python -u tools/gemm_bench.py > $O/cfg10.txt 2>&1 || exit 5
echo "cfg10 done"
