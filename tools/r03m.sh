set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03m "tests/test_gpu_graph.py tests/test_gpu_train.py" || exit 1
for cfg in latent_vit hybrid_latent_vit image_vit_48; do
 for wc in 0 1; do
  FERVIT_WGRAD_CAPTURE=$wc timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03m_${cfg}_$wc.txt 2>&1 || { tail -5 gpurun_out/r03m_${cfg}_$wc.txt; exit 1; }
  echo "$cfg wcap=$wc $(tail -1 gpurun_out/r03m_${cfg}_$wc.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_ms_median"], d["final_loss"])')"
 done
done
