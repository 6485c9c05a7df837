cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/t.txt 2>&1; tail -2 gpurun_out/t.txt; grep -q failed gpurun_out/t.txt && { grep -E "^E " gpurun_out/t.txt | head -20; exit 1; }
cd tools
for c in 8 5; do FERVIT_GEMM_CFG=$c GB_ONLY=wgrad timeout -k 10 200 python gemm_bench.py 2>&1 | grep -v amdgpu.ids >> ../gpurun_out/gb10.txt || exit 1; done
timeout -k 10 200 python gemm_bench.py 2>&1 | grep -v amdgpu.ids >> ../gpurun_out/gb10.txt || exit 1
cat ../gpurun_out/gb10.txt
cd .. && timeout -k 10 300 python bench.py > gpurun_out/bench.txt 2>&1; tail -3 gpurun_out/bench.txt
