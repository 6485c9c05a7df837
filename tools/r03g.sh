set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/micro/hash_rate > gpurun_out/r03g_hash_rate.txt 2>&1 || exit 1
cat gpurun_out/r03g_hash_rate.txt
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r03g_bench.txt 2>&1 || { tail -5 gpurun_out/r03g_bench.txt; exit 1; }
tail -1 gpurun_out/r03g_bench.txt | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03g_tl -o run \
  -- python3 bench.py --steps 8 --warmup 3 --probe-steps 0 --no-cpu-baseline --no-traffic > gpurun_out/r03g_tl.log 2>&1 || { tail -5 gpurun_out/r03g_tl.log; exit 1; }
python3 tools/timeline.py gpurun_out/r03g_tl/run_kernel_trace.csv 5 > gpurun_out/r03g_timeline.txt; head -50 gpurun_out/r03g_timeline.txt
