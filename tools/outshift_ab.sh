#!/bin/bash
# Inputs all at one 16-B offset: the outshift kernels (realign the outputs) against the
# unaligned-load form (SOSX_*_OUTSHIFT=0 SOSX_REALIGN_UNALIGNED=1), prefix and fold,
# P inputs of 16Mi fp32, interleaved twice (tools/misaligned_probe.py).  Output on stdout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for r in 1 2; do
  for np in ${NPS:-1 2 3 4 8}; do
    for o in 1 0; do
      for what in prefix fold; do
        [ "$what" = fold ] && [ "$np" -lt 2 ] && continue
        SOSX_PREFIX_OUTSHIFT=$o SOSX_FOLD_OUTSHIFT=$o SOSX_REALIGN_UNALIGNED=$((o ? 5 : 1)) timeout -k 10 120 \
          python3 tools/misaligned_probe.py --$what --np "$np" --only all+4,all+8 2> /tmp/ab.err > /dev/null || { tail -5 /tmp/ab.err; exit 1; }
        grep -v amdgpu.ids /tmp/ab.err | sed "s/^/np=$np outshift=$o /"
      done
    done
  done
done
