set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "attention" -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/tests_r03at.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_r03at.txt; [ $rc -eq 0 ] || exit $rc
B=$GRAFT_REPO_ROOT/fer-vit_amd/fervit/libfervit_base.so
for i in 1 2 3; do
  ATT_TAG=new timeout -k 10 120 python -u tools/attn_time.py 2>/dev/null || exit 1
  FERVIT_LIB=$B ATT_TAG=base timeout -k 10 120 python -u tools/attn_time.py 2>/dev/null || exit 1
done
for v in "A=1" "FERVIT_LIB=$B" "A=1" "FERVIT_LIB=$B"; do
  env $v timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-traffic --probe-steps 1 > gpurun_out/r03at.txt 2>&1 || { tail -5 gpurun_out/r03at.txt; exit 1; }
  echo "[${v:0:10}] vitb $(tail -1 gpurun_out/r03at.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_ms_median"], d["final_loss"])')"
done
