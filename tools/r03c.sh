set -o pipefail
bash tools/gpu_tests.sh r03c "tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_graph.py tests/test_gpu_rccl.py" "multi_unit or head_dropout or reference_train or stale or pending or lr_scheduler or rccl or persistent_work or graph_replay or every_tile or epilogue_kinds or linear_fwd_dgrad or many_tiles" || exit 1
cd $GRAFT_REPO_ROOT
GB_ONLY=gate,mul,res_fc2,store_qkv,plain_fc1,wgrad timeout -k 10 200 python -u tools/gemm_cases_bench.py > gpurun_out/r03c_gemm.txt 2>&1 || exit 1
FERVIT_GEMM_CFG=10 GB_TAG=pp GB_ONLY=gate,mul,res_fc2,store_qkv,plain_fc1 timeout -k 10 200 python -u tools/gemm_cases_bench.py >> gpurun_out/r03c_gemm.txt 2>&1 || exit 1
cat gpurun_out/r03c_gemm.txt
