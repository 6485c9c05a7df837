# fc1 weight gradient (MN x MN operands, split-K) under each 256-wide tile configuration
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for c in 5 4 8 9 1 0; do
  (cd tools && GB_ONLY=wgrad GB_CFG=$c timeout -k 10 120 python -u gemm_bench.py 2>&1 | grep -v amdgpu.ids) \
    | tee -a gpurun_out/${1:-x}_wgrad_cfg.txt || exit 1
done
