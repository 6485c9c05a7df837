set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in "A=1" "FERVIT_REDUCE_MAX_KB=8192" "A=1" "FERVIT_REDUCE_MAX_KB=8192" "A=1" "FERVIT_REDUCE_MAX_KB=8192"; do
  env $v timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-traffic --probe-steps 1 > gpurun_out/r03av.txt 2>&1 || { tail -5 gpurun_out/r03av.txt; exit 1; }
  echo "[$v] vitb $(tail -1 gpurun_out/r03av.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_ms_median"], d["final_loss"])')"
done
