set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03n "tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_graph.py tests/test_gpu_train.py tests/test_gpu_hybrid.py" "wgrad or latent or image_vit_48 or graph or epoch or hybrid or reference" || exit 1
O=gpurun_out/r03n_lat_gemm.txt; : > $O
export GB_ONLY=qkv_wgrad,out_wgrad,fc1_wgrad,fc2_wgrad,wgrad_group
for sp in 0 1 2; do
FERVIT_WG_SPLITS=$sp GB_TAG=sp$sp timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || { tail -5 $O; exit 1; }
done
FERVIT_WG_NST3=1 GB_TAG=nst3 timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || { tail -5 $O; exit 1; }
grep -v amdgpu.ids $O | grep -v "layer sum"
for cfg in latent_vit image_vit_48; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03n_$cfg.txt 2>&1 || { tail -5 gpurun_out/r03n_$cfg.txt; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/r03n_$cfg.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"
done
