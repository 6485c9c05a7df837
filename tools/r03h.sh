set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp FERVIT_PROBE_ALL=1
timeout -k 10 300 python -u bench.py --config latent_vit --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r03h_lat.txt 2>&1 || { tail -5 gpurun_out/r03h_lat.txt; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > gpurun_out/r03h_vitb.txt 2>&1 || { tail -5 gpurun_out/r03h_vitb.txt; exit 1; }
grep -v "^{" gpurun_out/r03h_lat.txt | tail -40; tail -1 gpurun_out/r03h_lat.txt | cut -c1-200
grep -v "^{" gpurun_out/r03h_vitb.txt | tail -20
