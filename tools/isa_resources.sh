#!/bin/bash
# Per-kernel register / scratch / spill counts of every step-kernel instance (compile-time, no GPU):
# each build part of fw_kernels.hip compiled with -Rpass-analysis=kernel-resource-usage, in parallel.
# Usage: tools/isa_resources.sh > profiles/r05_isa_resources.txt
SRC=$(cd "$(dirname "$0")/.." && pwd)/tum_adlr_deep_reinforcement_learning_amd/csrc/fw_kernels.hip
W=$(mktemp -d)
for p in 1 2 3 4 5 6; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -DFW_PART=$p -c "$SRC" \
    -o "$W/p$p.o" -Rpass-analysis=kernel-resource-usage > "$W/p$p.txt" 2>&1 &
done
# the rollout-side kernels too (k_policy_mfma, k_merge_update16, k_gae, ...)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -c "$(dirname "$SRC")/fw_rollout.hip" \
  -o "$W/pr.o" -Rpass-analysis=kernel-resource-usage > "$W/pr.txt" 2>&1 &
wait
echo "# gfx950 resource usage per kernel instance (hipcc -Rpass-analysis=kernel-resource-usage, $(date -u +%F))"
echo "# vgpr/agpr: registers per lane (vgpr+agpr > 256 uses the AGPR half; 512 = one wave per SIMD);"
echo "# scratch: bytes per lane (a kernel that calls env_step_noinl includes the call frame); vspill/sspill: spilled VGPRs / SGPRs"
cat "$W"/p*.txt | grep remark | sed -e 's/.*remark: *//; s/ \[-Rpass.*//' | \
  awk '/Function Name/{n=$3; sub(/_ZN12_GLOBAL__N_1[0-9]+/,"",n); sub(/EEvPK.*/,"",n)} /^VGPRs:/{v=$2} /^AGPRs/{a=$2}
       /ScratchSize/{s=$3} /^VGPRs Spill/{vs=$3} /^SGPRs Spill/{ss=$3} /^Occupancy/{o=$3}
       /LDS Size/{if (n ~ /^k_/ || n ~ /noinl/) printf "%-58s vgpr %4s agpr %4s scratch %5s vspill %4s sspill %4s occ %s\n", n, v, a, s, vs, ss, o}' | sort -u
rm -rf "$W"
