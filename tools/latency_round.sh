#!/bin/bash
# Small-message latency table: tools/latency_check.py under tools/oshrun
# for P = 2, 4, 8 PEs on this box's GPU (p2p transport), device-heap and host-heap
# operands, and SOS's own CPU recdbl_sw on the same P processes.  Output:
# gpurun_out/latency_<tag>/P<P>.txt.  Each P has its own time limit; stops at a failure.
set -u
tag=${1:-r3}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/latency_$tag
mkdir -p "$out"
export SHMEMX_TRANSPORT=p2p SHMEMX_DEVICE_HEAP_SIZE=256M SHMEMX_STAGE_BYTES=64M SHMEMX_DEVICE=0
for P in ${PES:-2 4 8}; do
    echo "=== P=$P $(date +%T)"
    timeout -k 10 240 python3 tools/oshrun -np "$P" --timeout 220 python3 tools/latency_check.py ${LAT_ARGS:-} > "$out/P$P.txt" 2> "$out/P$P.err"
    rc=$?
    echo "=== P=$P rc=$rc $(date +%T)"
    cat "$out/P$P.txt"
    [ $rc -eq 0 ] || { tail -20 "$out/P$P.err"; exit $rc; }
done
