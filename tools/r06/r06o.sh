#!/bin/bash
# r06o: full GPU suite after the attention changes (tail trim, backward lane table, dot2 Dq, no SLP), smoke,
# the default ViT-B bench, then the attention stamp timeline of the stamp build
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06o && export TMPDIR=/tmp
O=gpurun_out/r06o
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.txt 2>&1; rc=$?
echo "gpu tests rc=$rc $(grep -c PASSED $O/gpu_tests.txt) passed $(grep -c FAILED $O/gpu_tests.txt) failed"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 5
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 6; tail -1 $O/bench.json | cut -c1-300
FERVIT_LIB=$GRAFT_REPO_ROOT/fer-vit_amd/fervit/libfervit_st.so timeout -k 10 300 python -u tools/attn_stamps.py > $O/attn_stamps.txt 2>&1 || exit 7
