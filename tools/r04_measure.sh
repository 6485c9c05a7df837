# Round-4 measurements: bf16 parity errors (gates of tests/test_gpu_models.py), the small configs'
# bench lines with the step graph on and off, and the fc1 weight-gradient tile-config sweep.
set -o pipefail
TAG=${1:-r04x}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bf16_parity_measure.py > gpurun_out/${TAG}_bf16_parity.json 2> gpurun_out/${TAG}_bf16_parity.err \
  || { tail -20 gpurun_out/${TAG}_bf16_parity.err; exit 1; }
cat gpurun_out/${TAG}_bf16_parity.json
for cfg in hybrid_latent_vit expression_aware_vit; do
  for gr in off on; do
    timeout -k 10 300 python -u bench.py --config $cfg --graph $gr --steps 100 --warmup 10 --no-cpu-baseline --no-traffic \
      > gpurun_out/${TAG}_bench_${cfg}_graph_${gr}.json 2> gpurun_out/${TAG}_bench_${cfg}_graph_${gr}.err \
      || { tail -20 gpurun_out/${TAG}_bench_${cfg}_graph_${gr}.err; exit 1; }
    echo "$cfg graph=$gr $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d.get('launch'))" gpurun_out/${TAG}_bench_${cfg}_graph_${gr}.json)"
  done
done
bash tools/wgrad_cfg_sweep.sh $TAG
