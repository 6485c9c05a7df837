#!/bin/bash
# r06j: kernel-trace statistics of every bench configuration at HEAD (rocprofv3 --kernel-trace --stats)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06j && export TMPDIR=/tmp
for cfg in vit_base_224 latent_vit hybrid_latent_vit expression_aware_vit image_vit_48; do
  d=gpurun_out/r06j/prof_$cfg
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --config $cfg \
    --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 tools/prof_csv_summary.py "$f" 26 30 > gpurun_out/r06j/summary_$cfg.txt
  tail -1 $d.log | cut -c1-200
done
