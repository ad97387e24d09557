#!/bin/bash
# Stream-signalled p2p executor calls: the entry boundary on the host (the default) against
# queued as the first signalling step (SHMEMX_P2P_ENTRY=device), interleaved three times,
# P = 2 and 4 on this box's one GPU, device operands on the executor (tools/latency_check.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/entry_ab
mkdir -p "$out"
export SHMEMX_TRANSPORT=p2p SHMEMX_DEVICE_HEAP_SIZE=256M SHMEMX_STAGE_BYTES=64M SHMEMX_DEVICE=0
export SHMEMX_SMALL_DEVICE=0 SHMEMX_P2P_SIGNAL=stream
for P in ${PES:-2 4}; do
  for k in 1 2 3; do
    for entry in host device; do
      SHMEMX_P2P_ENTRY=$entry timeout -k 10 200 python3 tools/oshrun -np "$P" --timeout 180 python3 tools/latency_check.py --legs dev > "$out/P${P}_${entry}_$k.txt" 2> "$out/P${P}_${entry}_$k.err" || { tail -5 "$out/P${P}_${entry}_$k.err"; exit 1; }
      echo "P=$P round $k entry $entry:"; grep "dev" "$out/P${P}_${entry}_$k.txt"
    done
  done
done
