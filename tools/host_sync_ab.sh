#!/bin/bash
# Host-signalled p2p executor calls (SHMEMX_P2P_SIGNAL=host, the default across GPUs):
# a round's drain serving as the next completion point (the default) against a separate
# drain and completion (SOSX_TEST_SEPARATE_SYNCS=1, test build), interleaved three times,
# P = 2 and 4 on this box's one GPU, device operands on the executor (tools/latency_check.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/host_sync_ab
mkdir -p "$out"
export SHMEMX_TRANSPORT=p2p SHMEMX_DEVICE_HEAP_SIZE=256M SHMEMX_STAGE_BYTES=64M SHMEMX_DEVICE=0
export SHMEMX_SMALL_DEVICE=0 SHMEMX_P2P_SIGNAL=host SOSX_LIBRARY=$(pwd)/tests/fakerccl/libsos_amd_fakerccl.so
for P in ${PES:-2 4}; do
  for k in 1 2 3; do
    for sep in 0 1; do
      SOSX_TEST_SEPARATE_SYNCS=$sep timeout -k 10 200 python3 tools/oshrun -np "$P" --timeout 180 python3 tools/latency_check.py --legs dev > "$out/P${P}_sep${sep}_$k.txt" 2> "$out/P${P}_sep${sep}_$k.err" || { tail -5 "$out/P${P}_sep${sep}_$k.err"; exit 1; }
      echo "P=$P round $k separate $sep:"; grep "dev" "$out/P${P}_sep${sep}_$k.txt"
    done
  done
done
