cd $GRAFT_REPO_ROOT/tools && mkdir -p ../gpurun_out
for d in 0 1 2 3 4 5 7 8 15; do for c in 0 1; do FERVIT_GEMM_DBG=$d FERVIT_GEMM_CFG=$c GB_ONLY=fc2 timeout -k 10 100 python gemm_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/dbg$d /" >> ../gpurun_out/dbg.txt || exit 1; done; done
cat ../gpurun_out/dbg.txt
