# Round-4 profile set: GPU tests, the default bench line (with PMC traffic), a rocprofv3 kernel-trace
# summary of a short bench run, the other configs' bench lines, SQ counters of the attention kernels.
set -o pipefail
TAG=${1:-r04x}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu_suite.sh $TAG tests bench prof || exit 1
python3 tools/timeline.py gpurun_out/${TAG}_prof/run_kernel_trace.csv 5 > gpurun_out/${TAG}_two_stream_timeline.txt 2>&1 || true
head -4 gpurun_out/${TAG}_two_stream_timeline.txt
for cfg in latent_vit image_vit_48 hybrid_latent_vit expression_aware_vit; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 > gpurun_out/${TAG}_bench_$cfg.json \
    2> gpurun_out/${TAG}_bench_$cfg.err || { tail -5 gpurun_out/${TAG}_bench_$cfg.err; exit 1; }
  echo "$cfg $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d.get('step_mfma_frac'))" gpurun_out/${TAG}_bench_$cfg.json)"
done
ATTN_CASE=fwd bash tools/pmc_sq.sh ${TAG}_attnfwd attn_once.py attn_fwd_pers SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES
bash tools/pmc_sq.sh ${TAG}_attnbwd attn_once.py attn_bwd_pers SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES
