#!/bin/bash
# r06i: split target of the small MN x MN weight gradient (out_proj, 9 tiles of 256^2): 224 (shipped) vs 144 / 108 / 72
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06i && export TMPDIR=/tmp
O=gpurun_out/r06i
for rep in 1 2; do for t in 224 144 108 72; do
  (cd tools && FERVIT_WGRAD_TGT_SMALL=$t GB_ONLY="out wgrad" timeout -k 10 120 python -u gemm_bench.py 2>&1 | grep -v amdgpu.ids) \
    | sed "s/^/[tgt $t] /" >> $O/gemm.txt || exit 1
done; done
cat $O/gemm.txt
timeout -k 10 900 python -u tools/step_ab.py --config vit_base_224 --rounds 5 --steps 10 base env:FERVIT_WGRAD_TGT_SMALL=144 \
  env:FERVIT_WGRAD_TGT_SMALL=108 env:FERVIT_WGRAD_TGT_SMALL=72 > $O/step_ab.txt 2>&1 || exit 2
tail -6 $O/step_ab.txt
