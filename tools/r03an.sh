set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_reduce_defer.py tests/test_gpu_models.py tests/test_gpu_hybrid.py -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/tests_r03an.txt 2>&1
rc=$?; tail -4 gpurun_out/tests_r03an.txt; [ $rc -eq 0 ] || exit $rc
for v in "A=1" "FERVIT_REDUCE_DEFER=0" "A=1" "FERVIT_REDUCE_DEFER=0"; do
  env $v timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-traffic --probe-steps 1 > gpurun_out/r03an.txt 2>&1 || { tail -5 gpurun_out/r03an.txt; exit 1; }
  echo "[$v] vitb $(tail -1 gpurun_out/r03an.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_ms_median"])')"
  for cfg in latent_vit hybrid_latent_vit expression_aware_vit image_vit_48; do
    env $v timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03an_$cfg.txt 2>&1 || { tail -5 gpurun_out/r03an_$cfg.txt; exit 1; }
    echo "[$v] $cfg $(tail -1 gpurun_out/r03an_$cfg.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
