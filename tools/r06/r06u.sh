#!/bin/bash
# r06u: gemm_bf16_kernel (128x64 / 128x128 / 256^2 double-buffered tiles: the small-token configurations) with
# alternating fragment sets: GEMM tests, then interleaved A/B against HEAD on the hybrid, latent and ImageViT-48 steps
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
KT="gemm" bash tools/lib_ab.sh r06u tests || exit 1
for c in hybrid_latent_vit latent_vit image_vit_48 expression_aware_vit; do
  CFG=$c REPS=3 bash tools/lib_ab.sh r06u_$c bench || exit 1
done
