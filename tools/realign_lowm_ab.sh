#!/bin/bash
# The realigning fold/prefix with few incongruent inputs: the DPP form (the default below
# SOSX_REALIGN_UNALIGNED = 5) against the unaligned-load form forced (=1).  Prefix: input 0
# at +4 B at P = 8 and P = 4 (and P = 4 mixed), interleaved twice; fold: tools/realign_ab.py
# on m1..m4 with the product forced to the unaligned form beside the DPP variant (3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for r in 1 2; do
  for u in 5 1; do
    SOSX_REALIGN_UNALIGNED=$u timeout -k 10 120 python3 tools/misaligned_probe.py --prefix --only input0+4 2> /tmp/lm.err > /dev/null || { tail -5 /tmp/lm.err; exit 1; }
    grep -v amdgpu.ids /tmp/lm.err | sed "s/^/np=8 ul_min=$u /"
    SOSX_REALIGN_UNALIGNED=$u timeout -k 10 120 python3 tools/misaligned_probe.py --prefix --np 4 --only input0+4,mixed 2> /tmp/lm.err > /dev/null || { tail -5 /tmp/lm.err; exit 1; }
    grep -v amdgpu.ids /tmp/lm.err | sed "s/^/np=4 ul_min=$u /"
  done
done
SOSX_REALIGN_UNALIGNED=1 timeout -k 10 300 python3 tools/realign_ab.py --rounds 2 --only 3 --layouts m1,m2,m3,m4 2>&1 | grep -v "amdgpu.ids\|^{"
