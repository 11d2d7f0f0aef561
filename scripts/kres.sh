#!/bin/bash
# Print VGPR / SGPR / occupancy / scratch per kernel of rt_kernels.hip (compile-only).
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -c "$(dirname $0)/../mini-opencl-raytracer_amd/csrc/rt_kernels.hip" -o /tmp/rt_kres.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | python3 -c "
import sys,re
cur=None
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur=m.group(1); print(); print(cur[:70], end=' ')
    for k in ('VGPRs:','SGPRs:','ScratchSize \[bytes/lane\]:','Occupancy \[waves/SIMD\]:'):
        m=re.search(k+r' (\d+)',l)
        if m: print(k.split()[0].strip(':'), m.group(1), end=' ')
print()"
