#!/bin/bash
# kernel resource usage (VGPRs, spills, LDS, occupancy) of one HIP source, gfx950
# usage: profiles/resusage.sh speedy-ml-1_amd/csrc/sml_dynamics.hip
src=$(readlink -f "$1")
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -c "$src" -o /tmp/_ru.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed -n 's/.*remark: *//p' | awk '
/Function Name/ {if (name) print line; name=$3; line=name; next}
/VGPRs:|AGPRs:|Spill|LDS Size|Occupancy|ScratchSize/ {sub(/ \[-Rpass.*/, ""); gsub(/ +/, " "); line=line " | " $0}
END {print line}' | c++filt | sed 's/(anonymous namespace):://'
