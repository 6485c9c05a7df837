set -o pipefail
cd "$GRAFT_REPO_ROOT/tools" && mkdir -p ../gpurun_out
for d in 0 4; do echo "== dbg $d"; FERVIT_GEMM_DBG=$d timeout -k 10 150 python -u gemm_ksweep.py 2>&1 | grep -v amdgpu.ids || exit 1; done | tee ../gpurun_out/dbg_$1.txt
