# One GPU call: the store-operand padding (csrc/store_hazard_pad.py) against the unpadded build
# (fer-vit_amd/fervit/libfervit_nopad.so, make PAD_W=0): the fold tests, the 128^2 residual-GEMM
# repeat stress on both libraries, and interleaved short bench runs on both. usage: bash tools/pad_ab.sh <tag>
set -o pipefail
TAG=${1:-pad}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/fer-vit_amd/fervit
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider --timeout 150 \
  --timeout-method thread -k "fold or row_tile" > gpurun_out/${TAG}_ktest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_ktest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_ktest.txt
for lib in libfervit.so libfervit_nopad.so; do
  FERVIT_LIB=$L/$lib GD_STRESS=${REPS:-150} timeout -k 10 400 python -u tools/gemm_determinism.py 2>&1 \
    | grep -v amdgpu.ids | sed "s/^/[$lib] /" | tee -a gpurun_out/${TAG}_stress.txt | tail -3 || exit 1
done
for rep in 1 2 3; do for lib in libfervit.so libfervit_nopad.so; do
  FERVIT_LIB=$L/$lib timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic \
    2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$lib]', d['ms_per_step'], d['step_ms_median'], d['roofline']['frac'], d['roofline'].get('frac_in_step'))" \
    | tee -a gpurun_out/${TAG}_bench_ab.txt || exit 1
done; done
