#!/bin/bash
# usage: tools/kres.sh <kernel .hip> [name-substring]: hipcc resource usage (VGPRs, spills) per kernel
cd /root/repo/ggml-imax_amd && /opt/rocm/bin/hipcc -O3 -DNDEBUG -fPIC -std=c++17 --offload-arch=gfx950 -fvisibility=hidden \
  -I../include -Icsrc/kernels -c "$1" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -E "error|Name|VGPRs|AGPRs|Spill" | grep -A4 "error\|${2:-.}" | grep -E "error|Name|Spill|VGPRs:|AGPRs:"
