cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/t.txt 2>&1; tail -2 gpurun_out/t.txt; grep -q failed gpurun_out/t.txt && { grep -E "^E |^FAILED" gpurun_out/t.txt | head -20; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench.txt 2>&1; tail -1 gpurun_out/bench.txt | cut -c1-300
export TMPDIR=/tmp; timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4 -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof4.log 2>&1; tail -1 gpurun_out/prof4.log | cut -c1-100
