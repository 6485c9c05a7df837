# One GPU call: a build A/B. The in-tree library (fer-vit_amd/fervit/libfervit.so) against another
# build in the same directory ($BASE, default libfervit_base.so): the GPU tests matching $KT on the
# in-tree library, then interleaved GEMM microbenchmarks ($GB_ONLY cases) and short bench runs on both.
# usage: [KT=...] [GB_ONLY=...] [BASE=lib.so] [REPS=3] [CFG=bench config] [BSTEPS=30] bash tools/lib_ab.sh <tag> [tests] [gbench] [abench] [bench]
set -o pipefail
TAG=${1:-ab}; shift
STEPS=${*:-tests gbench bench}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/fer-vit_amd/fervit
LIBS="libfervit.so ${BASE:-libfervit_base.so}"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 \
        --timeout-method thread -k "${KT:-gemm}" > gpurun_out/${TAG}_ktest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_ktest.txt; exit 1; }
      tail -2 gpurun_out/${TAG}_ktest.txt ;;
    gbench)
      for rep in 1 2; do for lib in $LIBS; do
        (cd tools && FERVIT_LIB=$L/$lib GB_ONLY="${GB_ONLY:-}" timeout -k 10 300 python -u gemm_bench.py 2>&1 | grep -v amdgpu.ids) \
          | sed "s/^/[$lib] /" | tee -a gpurun_out/${TAG}_gemm_ab.txt || exit 1
      done; done ;;
    abench)
      for rep in 1 2; do for lib in $LIBS; do
        (cd tools && FERVIT_LIB=$L/$lib timeout -k 10 300 python -u attn_bench.py 2>&1 | grep -v amdgpu.ids) \
          | sed "s/^/[$lib] /" | tee -a gpurun_out/${TAG}_attn_ab.txt || exit 1
      done; done ;;
    bench)
      for rep in $(seq ${REPS:-3}); do for lib in $LIBS; do
        FERVIT_LIB=$L/$lib timeout -k 10 300 python -u bench.py --config ${CFG:-vit_base_224} --steps ${BSTEPS:-30} --warmup 5 --no-cpu-baseline --no-traffic \
          2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$lib]', d['ms_per_step'], d['step_ms_median'], (d.get('roofline') or {}).get('frac'), (d.get('roofline') or {}).get('frac_in_step'))" \
          | tee -a gpurun_out/${TAG}_bench_ab.txt || exit 1
      done; done ;;
  esac
done
