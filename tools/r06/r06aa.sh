#!/bin/bash
# r06aa: fresh SQ counters of the attention kernels on the round-6 build (verdict r5 item 2: VALU : MFMA), one rocprofv3
# --pmc pass (8 SQ counters) over tools/attn_once.py (ViT-B/16 bs 256, N 197, 12 heads, p 0.1); then the kernel tests
# touched since the r06x suite (tile-config test with a single-K-step case)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06aa && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"
for k in attn_bwd_pers attn_fwd_occ; do
  timeout -k 10 150 bash tools/pmc_sq.sh r06aa_$k attn_once.py $k $C > gpurun_out/r06aa/pmc_$k.txt 2>&1 || exit 3
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "every_tile_config" > gpurun_out/r06aa/ktest.txt 2>&1; rc=$?; tail -2 gpurun_out/r06aa/ktest.txt; exit $rc
