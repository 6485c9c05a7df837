#!/bin/bash
# r06ak: validation of the round-6 build: full GPU suite, smoke, default ViT-B bench, kernel-trace summary of the bench
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06ak && export TMPDIR=/tmp
O=gpurun_out/r06ak
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.txt 2>&1; rc=$?
echo "gpu tests rc=$rc $(grep -c PASSED $O/gpu_tests.txt) passed $(grep -c FAILED $O/gpu_tests.txt) failed"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 5
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 6; tail -1 $O/bench.json | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --no-traffic > $O/prof.log 2>&1 || exit 7
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 tools/prof_csv_summary.py "$f" 26 30 > $O/kernel_summary.txt
