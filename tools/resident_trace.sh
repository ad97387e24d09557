#!/bin/bash
# Small-path phase times (SOSX_SMALL_TRACE) at P = 2 on one GPU, host-heap operands, with and
# without the resident executor.  Output: gpurun_out/res/trace_r<0|1>.err
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/res
export SHMEMX_TRANSPORT=p2p SHMEMX_DEVICE_HEAP_SIZE=256M SHMEMX_STAGE_BYTES=64M SHMEMX_DEVICE=0 LAT_REPS=500 SOSX_SMALL_TRACE=500
for r in 0 1; do
  SHMEMX_SMALL_RESIDENT=$r timeout -k 10 200 python3 tools/oshrun -np 2 --timeout 180 python3 tools/latency_check.py --legs host > gpurun_out/res/trace_r$r.txt 2> gpurun_out/res/trace_r$r.err || exit 1
done
echo done
