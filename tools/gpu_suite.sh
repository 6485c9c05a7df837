# One GPU call: the -m gpu suite, then the default bench line, then a rocprofv3 kernel-trace summary of
# a short bench run. usage: bash tools/gpu_suite.sh <tag> [tests|bench|prof ...]   (default: all three)
set -o pipefail
TAG=${1:-x}; shift
STEPS=${*:-tests bench prof}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    ktests)  # attention / GEMM / LayerNorm kernel tests only
      timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 150 \
        --timeout-method thread > gpurun_out/${TAG}_ktests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_ktests.txt; exit 1; }
      tail -2 gpurun_out/${TAG}_ktests.txt ;;
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 \
        --timeout-method thread ${TESTS_ARGS:-} > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
      tail -2 gpurun_out/${TAG}_tests.txt ;;
    bench)
      timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
        || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
      cut -c1-400 gpurun_out/${TAG}_bench.json ;;
    attn|gemm|ln)
      # A/B microbench: the in-tree library and fer-vit_amd/fervit/libfervit_base.so (if present), interleaved
      for rep in 1 2; do for lib in ${ABLIBS:-libfervit.so libfervit_base.so}; do
        [ -f fer-vit_amd/fervit/$lib ] || continue
        (cd tools && FERVIT_LIB=$GRAFT_REPO_ROOT/fer-vit_amd/fervit/$lib timeout -k 10 200 python -u ${s}_bench.py 2>&1 \
          | grep -v amdgpu.ids | sed "s/^/[$lib] /") | tee -a gpurun_out/${TAG}_${s}_ab.txt || exit 1
      done; done ;;
    astamps)
      FERVIT_LIB=$GRAFT_REPO_ROOT/fer-vit_amd/fervit/libfervit_st.so timeout -k 10 120 python -u tools/attn_stamps.py \
        > gpurun_out/${TAG}_attn_stamps.txt 2>&1 || { tail -20 gpurun_out/${TAG}_attn_stamps.txt; exit 1; }
      cat gpurun_out/${TAG}_attn_stamps.txt | grep -v amdgpu.ids ;;
    gstamps)
      for c in fc1gate fc1 fc2res; do
        FERVIT_LIB=$GRAFT_REPO_ROOT/fer-vit_amd/fervit/libfervit_st.so timeout -k 10 120 python -u tools/gemm_stamps.py $c \
          2>&1 | grep -v amdgpu.ids | sed "s/^/[$c] /" | tee -a gpurun_out/${TAG}_gemm_stamps.txt | grep -E "epilogue|prologue|steady" || exit 1
      done ;;
    cumask)  # which CUs / XCDs a CU-masked stream's workgroups land on
      timeout -k 10 120 ./tools/micro/cumask_probe > gpurun_out/${TAG}_cumask_probe.txt 2>&1 \
        || { tail -20 gpurun_out/${TAG}_cumask_probe.txt; exit 1; }
      cat gpurun_out/${TAG}_cumask_probe.txt ;;
    hybgate)  # bf16 errors of the hybrid / expression-aware tests (their BF16_GATES = 2x these)
      timeout -k 10 300 python -u tests/bf16_parity_measure.py --hybrid > gpurun_out/${TAG}_bf16_parity_hybrid.json \
        2> gpurun_out/${TAG}_bf16_parity_hybrid.err || { tail -20 gpurun_out/${TAG}_bf16_parity_hybrid.err; exit 1; }
      cat gpurun_out/${TAG}_bf16_parity_hybrid.json ;;
    ab)  # interleaved in-process step A/B of the variants in $AB (tools/step_ab.py)
      timeout -k 10 ${AB_TIMEOUT:-600} python -u tools/step_ab.py ${AB_ARGS:-} $AB > gpurun_out/${TAG}_step_ab.txt 2>&1 \
        || { tail -20 gpurun_out/${TAG}_step_ab.txt; exit 1; }
      grep -A40 "rounds x" gpurun_out/${TAG}_step_ab.txt ;;
    fault)  # round-4 fault diagnosis: ONE launch of the faulting build; must stay the last step of a call
      AMD_LOG_LEVEL=1 timeout -k 10 120 python -u tools/fault/run_fault.py > gpurun_out/${TAG}_fault.txt 2>&1
      echo "fault step rc=$?"; grep -v "^:3:" gpurun_out/${TAG}_fault.txt | tail -20; exit 0 ;;
    htrace)  # kernel + HIP API trace of a short bench run: compute-queue gaps vs host API calls
      timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d /tmp/${TAG}_htrace -o run -- \
        python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-traffic --probe-steps 1 > gpurun_out/${TAG}_htrace.json 2>&1 \
        || { tail -20 gpurun_out/${TAG}_htrace.json; exit 1; }
      f=$(find /tmp/${TAG}_htrace -name "*kernel_trace.csv" | head -1)
      [ -n "$f" ] && python3 tools/host_gaps.py "$(dirname $f)" 3 > gpurun_out/${TAG}_host_gaps.txt 2>&1
      ls -la $(dirname ${f:-/tmp/x}) >> gpurun_out/${TAG}_host_gaps.txt 2>&1
      head -40 gpurun_out/${TAG}_host_gaps.txt ;;
    wgcfg)  # weight-gradient GEMMs: the automatic config vs the 8-phase kernel (MT16 / MT32), interleaved runs
      for c in auto 8 9 auto 8 9; do
        if [ $c = auto ]; then unset GB_CFG; else export GB_CFG=$c; fi
        (cd tools && GB_ONLY=wgrad timeout -k 10 200 python -u gemm_bench.py 2>&1 | grep -v amdgpu.ids) \
          | tee -a gpurun_out/${TAG}_wgrad_cfg.txt || exit 1
      done; unset GB_CFG ;;
    gbench)  # GEMM microbenchmark cases whose name contains $GB_ONLY (tools/gemm_bench.py)
      (cd tools && GB_ONLY="${GB_ONLY:-}" timeout -k 10 300 python -u gemm_bench.py 2>&1 | grep -v amdgpu.ids) \
        > gpurun_out/${TAG}_gemm_bench.txt || { tail -20 gpurun_out/${TAG}_gemm_bench.txt; exit 1; }
      cat gpurun_out/${TAG}_gemm_bench.txt ;;
    ktest)  # the GPU tests whose name matches $KT (pytest -k)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$KT" \
        > gpurun_out/${TAG}_ktest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_ktest.txt; exit 1; }
      tail -5 gpurun_out/${TAG}_ktest.txt ;;
    smoke)  # __graft_entry__.smoke() on cuda:0
      timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${TAG}_smoke.txt 2>&1 \
        || { tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
      tail -3 gpurun_out/${TAG}_smoke.txt ;;
    configs)  # the other bench configurations (SURVEY 8(d) cfg 2, 4, 5 and the 48 px ImageViT)
      for c in latent_vit hybrid_latent_vit expression_aware_vit image_vit_48; do
        timeout -k 10 300 python -u bench.py --config $c --steps ${CFG_STEPS:-50} --warmup 10 --no-cpu-baseline \
          > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { tail -20 gpurun_out/${TAG}_bench_$c.err; exit 1; }
        cut -c1-240 gpurun_out/${TAG}_bench_$c.json
      done ;;
    determ)  # run-to-run and 256- vs 224-row bit equality of the residual-kind GEMM
      timeout -k 10 200 python -u tools/gemm_determinism.py > gpurun_out/${TAG}_determinism.txt 2>&1 \
        || { tail -20 gpurun_out/${TAG}_determinism.txt; exit 1; }
      grep -v amdgpu.ids gpurun_out/${TAG}_determinism.txt ;;
    fwdcc)  # two concurrent half-batch forwards vs sequential (tools/fwd_concurrency.py)
      timeout -k 10 300 python -u tools/fwd_concurrency.py > gpurun_out/${TAG}_fwd_concurrency.txt 2>&1 \
        || { tail -20 gpurun_out/${TAG}_fwd_concurrency.txt; exit 1; }
      grep -v amdgpu.ids gpurun_out/${TAG}_fwd_concurrency.txt ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
        python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/${TAG}_prof.json 2>&1 \
        || { tail -20 gpurun_out/${TAG}_prof.json; exit 1; }
      f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
      python3 tools/prof_csv_summary.py "$f" 19 40 > gpurun_out/${TAG}_kernel_summary.txt 2>&1 || true
      head -30 gpurun_out/${TAG}_kernel_summary.txt ;;
  esac
done
