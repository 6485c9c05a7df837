# SQ counters of the attention kernels (one pass per counter group). usage: bash tools/attn_pmc.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-a}
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_${TAG}_$i -o run -- python3 tools/attn_once.py > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_ attn_ | tee gpurun_out/pmc_${TAG}_summary.txt
