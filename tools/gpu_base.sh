# Baseline measurements: GEMM cases with / without epilogue, SQ counters per epilogue kind, a
# kernel trace of the bench for tools/timeline.py.  usage: bash tools/gpu_base.sh <tag> [pmc cases]
set -o pipefail
TAG=${1:-base}
PMC_CASES=${2:-"gate res_fc2 mul"}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 python -u tools/gemm_cases_bench.py > $O/gemm_cases.txt 2>&1 || { tail -20 $O/gemm_cases.txt; exit 1; }
FERVIT_GEMM_DBG=4 timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O/gemm_cases.txt 2>&1 || { tail -20 $O/gemm_cases.txt; exit 1; }
cat $O/gemm_cases.txt
for c in $PMC_CASES; do
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    GEMM_CASE=$c timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${c}_$i -o run -- python3 tools/gemm_case.py > $O/pmc_${c}_$i.log 2>&1 || { tail -5 $O/pmc_${c}_$i.log; exit 1; }
  done
  python3 tools/pmc_summary.py $O/pmc_${c}_ gemm_ > $O/pmc_${c}_summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log
python3 tools/timeline.py $O/prof/run_kernel_trace.csv 5 > $O/timeline.txt && head -30 $O/timeline.txt
