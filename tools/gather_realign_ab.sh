#!/bin/bash
# The p2p gather with sources at +4 / +8 / +12 bytes: the DPP shape (SOSX_GATHER_REALIGN=0)
# against one unaligned load per vector (=2), interleaved twice; congruent for reference
# (tools/gather_bench.py, 7 segments x 64 MiB, one launch).  Output on stdout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for r in 1 2; do
  SOSX_GATHER_REALIGN=0 timeout -k 10 120 python3 tools/gather_bench.py --src-offset 0 2>/dev/null | sed "s/^/mode=0 /" || exit 1
  for off in 4 8 12; do
    for m in 0 2; do
      SOSX_GATHER_REALIGN=$m timeout -k 10 120 python3 tools/gather_bench.py --src-offset $off 2>/dev/null | sed "s/^/mode=$m /" || exit 1
    done
  done
done
