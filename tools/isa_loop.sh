#!/bin/bash
# Static instruction mix of k_env_step<float>'s RK loop (compile-only, no GPU).
# Usage: tools/isa_loop.sh [extra hipcc flags...]
set -e
SRC=$(cd "$(dirname "$0")/.." && pwd)/tum_adlr_deep_reinforcement_learning_amd/csrc/fw_kernels.hip
W=$(mktemp -d)
cd "$W"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize --save-temps "$@" -c "$SRC" -o k.o 2>/dev/null
S=$(ls *gfx950.s)
awk -v pat="${KPAT:-k_env_stepIfN2fw8GymX8CfgIfEELb0}" '$0 ~ "^_ZN12_GLOBAL__N_1[0-9]+" pat && /:/ {f=1} f&&/s_endpgm/{print; f=0} f' "$S" > env.s
grep -E "^\s+\.(vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size):" "$S" | tail -5 | tr -s ' ' | tr '\n' ' '
echo
# the RK loop = the depth-1 loop with the largest body
read H L0 L1 < <(awk '/^\.LBB[0-9_]+:/{lab=substr($1,3,length($1)-3); pos[lab]=NR} /Header=BB[0-9_]+ Depth=1/{match($0,/Header=BB[0-9_]+/); h=substr($0,RSTART+7,RLENGTH-7); last[h]=NR} END{best=0; for (h in last) if (h in pos && last[h]-pos[h]>best) {best=last[h]-pos[h]; bh=h} print bh, pos[bh], last[bh]}' env.s)
awk -v a="$L0" -v b="$L1" 'NR>=a && NR<=b+80' env.s > loop.s
echo "loop $H lines $L0..$L1"
printf "total %d  valu %d  v_mov %d  readlane %d  writelane %d  accvgpr %d  cndmask %d  salu %d  ds %d  waitcnt %d  f32arith %d  pk %d\n" \
  "$(grep -cE '^\s+[vsdg][a-z]' loop.s)" "$(grep -cE '^\s+v_' loop.s)" "$(grep -cE '^\s+v_mov_b(32|64)' loop.s)" \
  "$(grep -c v_readlane loop.s)" "$(grep -c v_writelane loop.s)" "$(grep -c v_accvgpr loop.s)" "$(grep -c v_cndmask loop.s)" \
  "$(grep -cE '^\s+s_' loop.s)" "$(grep -cE '^\s+ds_' loop.s)" "$(grep -c s_waitcnt loop.s)" \
  "$(grep -cE '^\s+v_(fma|fmac|fmamk|fmaak|mul|add|sub|subrev)_f32' loop.s)" "$(grep -cE '^\s+v_pk_' loop.s)"
cp loop.s /tmp/last_loop.s
cp env.s /tmp/last_env.s
rm -rf "$W"
