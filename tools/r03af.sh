set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in hybrid_latent_vit image_vit_48 latent_vit; do for v in "A=1" "FERVIT_WGRAD_SINGLE_GROUP=0" "A=1" "FERVIT_WGRAD_SINGLE_GROUP=0"; do
  env $v timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03af.txt 2>&1 || { tail -5 gpurun_out/r03af.txt; exit 1; }
  echo "$cfg [$v] $(tail -1 gpurun_out/r03af.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_ms_median"])')"
done; done
