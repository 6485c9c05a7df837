#!/bin/bash
# r06h: younger wave-row half at s_setprio 1 for the first k epilogue chunks (FER_EPI_PRIO = 1, 2, 4) vs shipped (0)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06h && export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/fer-vit_amd/fervit
O=gpurun_out/r06h
for rep in 1 2; do for lib in libfervit.so libfervit_ep1.so libfervit_ep2.so libfervit_ep4.so; do
  (cd tools && FERVIT_LIB=$L/$lib GB_ONLY="${GB_ONLY:-}" timeout -k 10 300 python -u gemm_bench.py 2>&1 | grep -v amdgpu.ids) \
    | sed "s/^/[$lib] /" >> $O/gemm_ab.txt || exit 1
done; done
echo gemm done
for rep in 1 2 3; do for lib in libfervit.so libfervit_ep1.so libfervit_ep2.so libfervit_ep4.so; do
  FERVIT_LIB=$L/$lib timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic 2>/dev/null | tail -1 \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$lib]', d['ms_per_step'], d['step_ms_median'])" >> $O/bench_ab.txt || exit 2
done; done
cat $O/bench_ab.txt
