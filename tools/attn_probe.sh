# Attention timing probe: p=0.1 / p=0 under the FERVIT_ATTN_DBG phase switches of the backward
# (attn_bwd_pers: 1 = no step math, 2 = no epilogue, 4 = idle producer). usage: bash tools/attn_probe.sh <tag> "0 1 2 4"
set -o pipefail
cd "$GRAFT_REPO_ROOT/tools" && mkdir -p ../gpurun_out
for d in ${2:-0 1 2 4}; do echo "== dbg $d"; FERVIT_ATTN_DBG=$d timeout -k 10 120 python -u attn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1; done | tee ../gpurun_out/attnprobe_$1.txt
