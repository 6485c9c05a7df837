set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_reduce_defer.py tests/test_gpu_models.py tests/test_gpu_hybrid.py tests/test_gpu_kernels.py -k "defer or model or hybrid or expression or wgrad_group or adamw or training" -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/tests_r03aq.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_r03aq.txt; [ $rc -eq 0 ] || exit $rc
for v in "A=1" "FERVIT_WG_TICKET_MEMSET=1" "A=1" "FERVIT_WG_TICKET_MEMSET=1"; do
  for cfg in latent_vit image_vit_48; do
    env $v timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03aq_$cfg.txt 2>&1 || { tail -5 gpurun_out/r03aq_$cfg.txt; exit 1; }
    echo "[$v] $cfg $(tail -1 gpurun_out/r03aq_$cfg.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
bash tools/r03ap.sh
