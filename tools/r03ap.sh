set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in 0 1 2 4; do for sp in 2 3 4 6; do
  FERVIT_WG_VARIANT=$v FERVIT_WG_SPLITS=$sp GB_ONLY=wgrad_group GB_TAG="v$v-sp$sp" timeout -k 10 120 python -u tools/gemm_latent_bench.py 2>/dev/null | grep wgrad_group || exit 1
done; done
