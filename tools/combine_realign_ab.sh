#!/bin/bash
# The realigning combine (`in` at another 16-B offset than inout) in its three shapes,
# SOSX_COMBINE_REALIGN = 0 (two aligned loads per lane) / 1 (DPP) / 2 (unaligned loads),
# interleaved twice, 512 MiB per operand (tools/misaligned_probe.py).  Output on stdout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for r in 1 2; do
  for m in 0 1 2; do
    SOSX_COMBINE_REALIGN=$m timeout -k 10 120 python3 tools/misaligned_probe.py 2> /tmp/cr.err > /dev/null || { tail -5 /tmp/cr.err; exit 1; }
    grep -v amdgpu.ids /tmp/cr.err | grep -v "+0:" | sed "s/^/mode=$m /"
  done
done
