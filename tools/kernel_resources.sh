#!/usr/bin/env bash
# Compact per-kernel resource report (VGPR/AGPR/scratch/occupancy/LDS) for one .hip file.
# usage: tools/kernel_resources.sh generativeaiexamples_amd/csrc/kernels/gemm.hip
f=$1
hipcc -O3 -std=c++17 --offload-arch=gfx950 -I"$(dirname "$0")/../generativeaiexamples_amd/csrc/include" -c "$f" -o /tmp/_kr.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed -n "s/.*remark: //p" | sed "s/ \[-Rpass.*//" | awk '
/Function Name:/ {name=$3}
/VGPRs:/ {v=$NF} /AGPRs:/ {a=$NF} /ScratchSize/ {s=$NF} /Occupancy/ {o=$NF}
/LDS Size/ {l=$NF; printf "%-90s vgpr=%-4s agpr=%-4s scratch=%-4s occ=%-3s lds=%s\n", substr(name,1,90), v, a, s, o, l}'
