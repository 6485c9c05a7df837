# Attention timing probe: p=0.1 / p=0 and the FERVIT_ATTN_DBG phase switches (1 = skip Dq, 2 = skip steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT/tools" && mkdir -p ../gpurun_out
for d in 0 2; do echo "== dbg $d"; FERVIT_ATTN_DBG=$d timeout -k 10 120 python -u attn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1; done | tee ../gpurun_out/attnprobe_$1.txt
