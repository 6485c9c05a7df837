set -o pipefail
cd "$GRAFT_REPO_ROOT/tools" && mkdir -p ../gpurun_out
for r in 1 2; do for v in gen fused; do echo "== $v"; if [ $v = gen ]; then export FERVIT_ATTN_GENERAL=1; else unset FERVIT_ATTN_GENERAL; fi
timeout -k 10 120 python -u attn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1; done; done | tee ../gpurun_out/attn_$1.txt
