#!/bin/bash
# r06g: phase stamps of the 8-phase GEMM main loop (diagnostic build libfervit_st.so; fixed stride so that WG 0's
# second tile is tile gridDim.x, the stamped one): fc1 GELU-gate kind (K 768), fc2 residual kind (K 3072)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06g && export TMPDIR=/tmp
for c in fc1gate fc2res; do
  FERVIT_FIXED_STRIDE=1 FERVIT_LIB=$GRAFT_REPO_ROOT/fer-vit_amd/fervit/libfervit_st.so timeout -k 10 120 \
    python -u tools/gemm_stamps.py $c > gpurun_out/r06g/stamps_$c.txt 2>&1 || exit 1
done
echo done
