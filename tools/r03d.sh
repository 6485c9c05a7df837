set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03d "tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_graph.py tests/test_gpu_rccl.py" "multi_unit or head_dropout or reference_train or stale or pending or lr_scheduler or rccl or persistent_work or graph_replay or every_tile or epilogue_kinds or linear_fwd_dgrad or many_tiles" || exit 1
O=gpurun_out/r03d_gemm.txt
timeout -k 10 200 python -u tools/gemm_cases_bench.py > $O 2>&1 || exit 1
FERVIT_GEMM_DBG=16 GB_TAG=old-split-order GB_ONLY=wgrad timeout -k 10 100 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
FERVIT_GEMM_CFG=10 GB_TAG=pp timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
cat $O
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r03d_bench.txt 2>&1 || { tail -5 gpurun_out/r03d_bench.txt; exit 1; }
tail -1 gpurun_out/r03d_bench.txt | cut -c1-400
