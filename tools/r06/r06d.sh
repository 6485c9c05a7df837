#!/bin/bash
# r06d: full GPU suite after the round-6 prune + pad-pass change, smoke, ViT-B bench
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06d && export TMPDIR=/tmp
O=gpurun_out/r06d
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.txt 2>&1; rc=$?
echo "gpu tests rc=$rc $(grep -c PASSED $O/gpu_tests.txt) passed $(grep -c FAILED $O/gpu_tests.txt) failed"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 5
for i in 1 2; do timeout -k 10 300 python -u bench.py > $O/bench_$i.json 2> $O/bench_$i.err || exit 6; tail -1 $O/bench_$i.json; done
