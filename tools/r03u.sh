set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/tests_r03u.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_r03u.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03u.txt 2>&1 || { tail -5 gpurun_out/smoke_r03u.txt; exit 1; }
tail -3 gpurun_out/smoke_r03u.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r03u_bench.txt 2>&1 || { tail -5 gpurun_out/r03u_bench.txt; exit 1; }
tail -1 gpurun_out/r03u_bench.txt | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03u_prof -o run \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r03u_prof.log 2>&1 || { tail -5 gpurun_out/r03u_prof.log; exit 1; }
python3 tools/prof_csv_summary.py gpurun_out/r03u_prof/run_kernel_stats.csv 27 40 > gpurun_out/r03u_summary.txt; head -30 gpurun_out/r03u_summary.txt
