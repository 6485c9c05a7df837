set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/tests_r03f.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_r03f.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03f.txt 2>&1 || { tail -5 gpurun_out/smoke_r03f.txt; exit 1; }
tail -2 gpurun_out/smoke_r03f.txt
O=gpurun_out/r03f_gemm.txt
export FERVIT_LIB=$PWD/fer-vit_amd/fervit/libfervit_exp.so
export FERVIT_GEMM_CFG=10 GB_ONLY=gate,mul,res_fc2,plain_fc1
GB_TAG=pp timeout -k 10 200 python -u tools/gemm_cases_bench.py > $O 2>&1 || exit 1
for d in 10 20 40; do
  FERVIT_GEMM_DBG=$((64 + (d << 8))) GB_TAG=pp-stagger-hi${d}k timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
done
FERVIT_GEMM_DBG=$((128 + (20 << 8))) GB_TAG=pp-stagger-odd20k timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
unset FERVIT_LIB FERVIT_GEMM_CFG GB_ONLY
cat $O
FERVIT_ATTN_DBG=1 timeout -k 10 120 python -u tools/attn_bench.py > gpurun_out/r03f_attn.txt 2>&1 || exit 1
FERVIT_ATTN_DBG=2 timeout -k 10 120 python -u tools/attn_bench.py >> gpurun_out/r03f_attn.txt 2>&1 || exit 1
cat gpurun_out/r03f_attn.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03f_lat -o run \
  -- python3 bench.py --config latent_vit --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03f_lat.log 2>&1 || { tail -5 gpurun_out/r03f_lat.log; exit 1; }
tail -1 gpurun_out/r03f_lat.log | cut -c1-300
python3 tools/prof_csv_summary.py gpurun_out/r03f_lat/run_kernel_stats.csv 28 40 > gpurun_out/r03f_lat_summary.txt; head -45 gpurun_out/r03f_lat_summary.txt
