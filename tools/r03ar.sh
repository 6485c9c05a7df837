set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_reduce_defer.py -k "wgrad_group or defer" -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/tests_r03ar.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_r03ar.txt; [ $rc -eq 0 ] || exit $rc
for v in "A=1" "FERVIT_WG_XCD=0" "A=1" "FERVIT_WG_XCD=0"; do
  env $v GB_ONLY=wgrad_group GB_TAG="$v" timeout -k 10 120 python -u tools/gemm_latent_bench.py 2>/dev/null | grep wgrad_group || exit 1
  for cfg in latent_vit image_vit_48 hybrid_latent_vit; do
    env $v timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03ar_$cfg.txt 2>&1 || { tail -5 gpurun_out/r03ar_$cfg.txt; exit 1; }
    echo "[$v] $cfg $(tail -1 gpurun_out/r03ar_$cfg.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
