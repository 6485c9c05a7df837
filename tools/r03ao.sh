set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03ao_prof -o run \
  -- python3 bench.py --config latent_vit --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03ao_prof.log 2>&1 || { tail -5 gpurun_out/r03ao_prof.log; exit 1; }
python3 tools/prof_csv_summary.py gpurun_out/r03ao_prof/run_kernel_stats.csv 26 40 > gpurun_out/r03ao_summary.txt; cat gpurun_out/r03ao_summary.txt
