set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03ag_hyb -o run \
  -- python3 bench.py --config hybrid_latent_vit --steps 20 --warmup 5 --probe-steps 0 --no-cpu-baseline > gpurun_out/r03ag_hyb.log 2>&1 || { tail -5 gpurun_out/r03ag_hyb.log; exit 1; }
python3 tools/prof_csv_summary.py gpurun_out/r03ag_hyb/run_kernel_stats.csv 28 40 > gpurun_out/r03ag_hyb_summary.txt; head -32 gpurun_out/r03ag_hyb_summary.txt
