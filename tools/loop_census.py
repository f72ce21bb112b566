#!/usr/bin/env python3
"""Static census of a step kernel's hot loops (CPU, no GPU): compiles one build part of fw_kernels.hip to
assembly, finds the kernel, and for its longest loops (backward branches) counts VALU instructions, AGPR moves
(v_accvgpr_read/write: VGPR overflow parked in the AGPR half) and scratch accesses (spills / stack).

  python tools/loop_census.py PART KERNEL_SUBSTRING [N_LOOPS]
  e.g. python tools/loop_census.py 2 k_env_stepIdN2fw8GymX8CfgIdEELb0ELi1E   (fp64 one-lane env step)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tum_adlr_deep_reinforcement_learning_amd", "csrc", "fw_kernels.hip")


def main():
    part, name = sys.argv[1], sys.argv[2]
    nloops = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    with tempfile.TemporaryDirectory() as w:
        asm = os.path.join(w, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize",
                        "-DFW_PART=" + part, "--cuda-device-only", "-S", SRC, "-o", asm], check=True)
        L = open(asm).read().split("\n")
    start = next(i for i, l in enumerate(L) if re.match(r"^_Z\w*" + re.escape(name) + r"\w*:", l))
    end = next(i for i in range(start + 1, len(L)) if L[i].strip().startswith("s_endpgm"))
    K = L[start:end + 1]
    labels = {m.group(1): i for i, l in enumerate(K) for m in [re.match(r"^(\.LBB\d+_\d+):", l)] if m}
    loops = []
    for i, l in enumerate(K):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))

    def census(seg):
        return {"valu": sum(1 for x in seg if x.strip().startswith("v_")),
                "accvgpr_moves": sum(1 for x in seg if "v_accvgpr" in x),
                "scratch": sum(1 for x in seg if "scratch_" in x),
                "salu_s_mov_b32": sum(1 for x in seg if x.strip().startswith("s_mov_b32"))}

    print("kernel", name, "instructions", len(K), "whole kernel", census(K))
    seen = []
    for a, b in sorted(loops, key=lambda x: x[1] - x[0], reverse=True):
        if any(abs(a - s) < 400 and abs(b - e) < 400 for s, e in seen):
            continue  # the same loop reached through another latch
        seen.append((a, b))
        print("loop lines %d-%d" % (a, b), census(K[a:b]))
        if len(seen) >= nloops:
            break


if __name__ == "__main__":
    main()
