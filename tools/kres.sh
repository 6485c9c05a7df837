#!/bin/bash
# usage: tools/kres.sh file.hip  -> per-kernel VGPR/AGPR/spill/LDS summary (gfx950)
f=$1; shift
cd "$(dirname "$f")" && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -I../../include "$@" -x hip -c "$(basename "$f")" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | sed -n 's/.*remark: //p' | awk '/Function Name/{n=$3} /VGPRs:/{v=$2} /AGPRs:/{a=$2} /VGPRs Spill/{s=$3} /ScratchSize/{sc=$3} /LDS Size/{l=$4; printf "%-90s v=%s a=%s spill=%s scratch=%s lds=%s\n", substr(n,1,90), v, a, s, sc, l}'
