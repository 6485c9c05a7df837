set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/r03i_lat_gemm.txt
GB_TAG=auto timeout -k 10 120 python -u tools/gemm_latent_bench.py > $O 2>&1 || { tail -5 $O; exit 1; }
for c in 2 6 7 1; do
  FERVIT_GEMM_CFG=$c GB_TAG=cfg$c timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || { tail -5 $O; exit 1; }
done
grep -v amdgpu.ids $O
