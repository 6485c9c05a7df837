set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03e "tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_graph.py tests/test_gpu_rccl.py" "attention or multi_unit or head_dropout or reference_train or stale or pending or lr_scheduler or rccl or persistent_work or graph_replay or every_tile or epilogue_kinds or linear_fwd_dgrad or many_tiles or pre_gate"
rc=$?; [ $rc -le 1 ] || exit $rc   # assertion failures (1) do not stop the measurements; a crash does
O=gpurun_out/r03e_gemm.txt
timeout -k 10 200 python -u tools/gemm_cases_bench.py > $O 2>&1 || exit 1
FERVIT_GEMM_DBG=16 GB_TAG=old-split-order GB_ONLY=wgrad timeout -k 10 100 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
FERVIT_GEMM_CFG=10 GB_TAG=pp timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
export FERVIT_LIB=$PWD/fer-vit_amd/fervit/libfervit_exp.so
GB_ONLY=gate,mul,res_fc2,store_qkv,plain_fc1 FERVIT_GEMM_DBG=32 GB_TAG=nostore timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
for d in 6 12 24; do
  GB_ONLY=gate,mul,res_fc2,store_qkv,plain_fc1 FERVIT_GEMM_DBG=$((64 + (d << 8))) GB_TAG=stagger${d}k timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
done
unset FERVIT_LIB
cat $O
timeout -k 10 120 python -u tools/attn_bench.py > gpurun_out/r03e_attn.txt 2>&1 || exit 1
FERVIT_ATTN_FWD_NOPIPE=1 timeout -k 10 120 python -u tools/attn_bench.py >> gpurun_out/r03e_attn.txt 2>&1 || exit 1
cat gpurun_out/r03e_attn.txt
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r03e_bench.txt 2>&1 || { tail -5 gpurun_out/r03e_bench.txt; exit 1; }
tail -1 gpurun_out/r03e_bench.txt | cut -c1-300
