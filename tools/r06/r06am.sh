#!/bin/bash
# r06am: SQ counters on the final round-6 build (one rocprofv3 --pmc pass of 8 SQ counters each): the attention kernels
# (tools/attn_once.py: ViT-B/16 bs 256, N 197, 12 heads, p 0.1) and the 8-phase GEMM's GELU-gate fc1 forward against its
# plain form (tools/gemm_once.py)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06am && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"
for k in attn_bwd_pers attn_fwd_occ; do
  timeout -k 10 150 bash tools/pmc_sq.sh r06am_$k attn_once.py $k $C > gpurun_out/r06am/pmc_$k.txt 2>&1 || exit 3
done
for c in fc1 fc1_gate; do
  GEMM_CASE=$c timeout -k 10 150 bash tools/pmc_sq.sh r06am_$c gemm_once.py gemm_8ph $C > gpurun_out/r06am/pmc_gemm_$c.txt 2>&1 || exit 4
done
cat gpurun_out/r06am/pmc_*.txt
