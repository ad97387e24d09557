#!/bin/bash
# The consumer-side acquire's price on small p2p executor calls:
# tools/latency_check.py on the test build of the library (tests/fakerccl/, compiled with
# SOSX_TEST_HOOKS), device-heap operands on the executor (SHMEMX_SMALL_DEVICE=0), with the
# protocol's acquire kernels on and off (SOSX_TEST_NO_ACQUIRE=1), interleaved three times,
# P = 2 and 4 on this box's one GPU (PES=...), stream signalling unless SIGNAL=host.
# Output: gpurun_out/acquire_cost${SIGNAL:+_$SIGNAL}/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/acquire_cost${SIGNAL:+_$SIGNAL}
mkdir -p "$out"
export SHMEMX_TRANSPORT=p2p SHMEMX_DEVICE_HEAP_SIZE=256M SHMEMX_STAGE_BYTES=64M SHMEMX_DEVICE=0
export SHMEMX_SMALL_DEVICE=0 SOSX_LIBRARY=$(pwd)/tests/fakerccl/libsos_amd_fakerccl.so
[ -n "${SIGNAL:-}" ] && export SHMEMX_P2P_SIGNAL=$SIGNAL
for P in ${PES:-2 4}; do
  for k in 1 2 3; do
    for skip in 0 1; do
      SOSX_TEST_NO_ACQUIRE=$skip timeout -k 10 200 python3 tools/oshrun -np "$P" --timeout 180 python3 tools/latency_check.py --legs dev > "$out/P${P}_skip${skip}_$k.txt" 2> "$out/P${P}_skip${skip}_$k.err" || { tail -5 "$out/P${P}_skip${skip}_$k.err"; exit 1; }
      echo "P=$P round $k acquire $((1 - skip)):"; grep "dev" "$out/P${P}_skip${skip}_$k.txt"
    done
  done
done
