set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03y "tests/test_gpu_kernels.py tests/test_gpu_models.py" "linear or every_tile or vit_base or many_tiles" || exit 1
O=gpurun_out/r03y.txt; : > $O
GB_ONLY=wgrad,wgrad_out,wgrad_qkv GB_TAG=auto timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-traffic --probe-steps 1 > gpurun_out/r03y_b.txt 2>&1 || { tail -5 gpurun_out/r03y_b.txt; exit 1; }
echo "new $(tail -1 gpurun_out/r03y_b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_ms_median"])')"
done
