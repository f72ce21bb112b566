#!/bin/bash
# Per-kernel register / scratch usage of libfwsim (compile-time, no GPU needed).
SRC=${1:-$(dirname "$0")/../tum_adlr_deep_reinforcement_learning_amd/csrc/fw_kernels.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -shared -o /tmp/_res.so "$SRC" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep remark | sed -e 's/.*remark: *//; s/ \[-Rpass.*//' | \
  awk '/Function Name/{n=$3; sub(/_ZN12_GLOBAL__N_1[0-9]+/,"",n); sub(/EEvPK.*/,"",n)} /^VGPRs:/{v=$2} /^AGPRs/{a=$2}
       /ScratchSize/{s=$3} /^VGPRs Spill/{vs=$3} /^SGPRs Spill/{ss=$3} /^Occupancy/{o=$3}
       /LDS Size/{printf "%-22s vgpr %4s agpr %4s scratch %5s vspill %4s sspill %4s occ %s\n", n, v, a, s, vs, ss, o}'
