#!/bin/bash
# Device-operand small-path calls with the fold awaiting the peers' posts on the GPU
# (SOSX_SMALL_GATE=1, the default) against the host waiting before the launch (=0),
# interleaved three times, P = 2 and 4 on this box's one GPU (tools/latency_check.py
# --legs dev, the small path's default SHMEMX_SMALL_DEVICE).  Output on stdout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/small_gate_ab
mkdir -p "$out"
export SHMEMX_TRANSPORT=p2p SHMEMX_DEVICE_HEAP_SIZE=256M SHMEMX_STAGE_BYTES=64M SHMEMX_DEVICE=0
for P in ${PES:-2 4}; do
  for k in 1 2 3; do
    for gate in 1 0; do
      SOSX_SMALL_GATE=$gate timeout -k 10 200 python3 tools/oshrun -np "$P" --timeout 180 python3 tools/latency_check.py --legs dev > "$out/P${P}_g${gate}_$k.txt" 2> "$out/P${P}_g${gate}_$k.err" || { tail -5 "$out/P${P}_g${gate}_$k.err"; exit 1; }
      echo "P=$P round $k gate $gate:"; grep "dev" "$out/P${P}_g${gate}_$k.txt"
    done
  done
done
