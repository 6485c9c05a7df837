#!/bin/bash
# r06f: token-assembly kernels (8-column forms) -- tests + lib A/B; tail layers' weight gradients on the compute stream
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06f && export TMPDIR=/tmp
O=gpurun_out/r06f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "tokens or step_in_backward or model_matches or train" > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/step_ab.py --config vit_base_224 --rounds 4 --steps 10 base tail:1 tail:2 > $O/tail_ab.txt 2>&1 || exit 3
tail -5 $O/tail_ab.txt
REPS=3 bash tools/lib_ab.sh r06f bench || exit 4
