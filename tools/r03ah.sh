set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/r03ah.txt; : > $O
for c in -1 3 11; do echo "[cfg $c]" >> $O; FERVIT_GEMM_CFG=$c timeout -k 10 120 python -u tools/gemm_small_kinds.py >> $O 2>&1 || exit 1; done
grep -v amdgpu.ids $O
bash tools/gpu_tests.sh r03ah "tests/test_gpu_hybrid.py tests/test_gpu_train.py" "hybrid or clip or adapter or cfg4 or cfg5" || exit 1
timeout -k 10 300 python -u bench.py --config hybrid_latent_vit --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03ah_h.txt 2>&1 || { tail -5 gpurun_out/r03ah_h.txt; exit 1; }
echo "hybrid $(tail -1 gpurun_out/r03ah_h.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_mfma_frac"])')"
