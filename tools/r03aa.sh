set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for t in 192 128 176 256 192 128 176 256; do
  FERVIT_GEMM_SPLIT_T256=$t timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-traffic --probe-steps 1 > gpurun_out/r03aa.txt 2>&1 || { tail -5 gpurun_out/r03aa.txt; exit 1; }
  echo "[t256=$t] $(tail -1 gpurun_out/r03aa.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_ms_median"])')"
done
