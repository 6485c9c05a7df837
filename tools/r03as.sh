set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/tests_r03as.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_r03as.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03as.txt 2>&1 || { tail -5 gpurun_out/smoke_r03as.txt; exit 1; }
tail -3 gpurun_out/smoke_r03as.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r03as_bench.txt 2>&1 || { tail -5 gpurun_out/r03as_bench.txt; exit 1; }
tail -1 gpurun_out/r03as_bench.txt | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03as_prof -o run \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r03as_prof.log 2>&1 || { tail -5 gpurun_out/r03as_prof.log; exit 1; }
python3 tools/prof_csv_summary.py gpurun_out/r03as_prof/run_kernel_stats.csv 27 40 > gpurun_out/r03as_summary.txt; head -16 gpurun_out/r03as_summary.txt
python3 tools/timeline.py gpurun_out/r03as_prof/run_kernel_trace.csv 5 > gpurun_out/r03as_timeline.txt; head -5 gpurun_out/r03as_timeline.txt
for cfg in latent_vit image_vit_48 hybrid_latent_vit expression_aware_vit; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 > gpurun_out/r03as_$cfg.txt 2>&1 || { tail -5 gpurun_out/r03as_$cfg.txt; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/r03as_$cfg.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_mfma_frac"], d["final_loss"])')"
done
