# A/B two libfervit builds on the bench configs (one box, interleaved): bash tools/ab_cfg.sh <tag> "<configs>"
set -o pipefail
TAG=${1:-abc}; CFGS=${2:-"hybrid_latent_vit latent_vit"}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do for L in fer-vit_amd/fervit/libfervit_base.so fer-vit_amd/fervit/libfervit.so; do for c in $CFGS; do
  FERVIT_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 240 python -u bench.py --config $c --steps 60 --warmup 10 --no-traffic --no-cpu-baseline --probe-steps 1 2>&1 | tail -1 \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L'.split('/')[-1], '$c', d['ms_per_step'])" || exit 1
done; done; done | tee gpurun_out/abcfg_$TAG.txt
