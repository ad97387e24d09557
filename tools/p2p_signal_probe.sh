#!/bin/bash
# p2p signalling modes on one GPU: team_check in stream mode (P=2, 3) as a correctness
# check, then the small/medium-call latency of both modes at P = 2, 4, 8.  Output under
# gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export SHMEMX_TRANSPORT=p2p SHMEMX_DEVICE_HEAP_SIZE=256M SHMEMX_STAGE_BYTES=64M SHMEMX_DEVICE=0
export SHMEMX_P2P_TIMEOUT=60 PYTHONPATH=$(pwd)
run() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    echo "=== $name" | tee -a gpurun_out/probe.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
    local rc=$?
    echo "=== $name rc=$rc" | tee -a gpurun_out/probe.log
    tail -n 4 "gpurun_out/$name.out"
    [ $rc -eq 0 ] || exit $rc
}
SHMEMX_P2P_SIGNAL=stream run tc2 200 python tools/oshrun -np 2 --timeout 180 python tests/team_check_pe.py
SHMEMX_P2P_SIGNAL=stream run tc3 200 python tools/oshrun -np 3 --timeout 180 python tests/team_check_pe.py
for P in 2 4 8; do
    for m in stream host; do
        SHMEMX_P2P_SIGNAL=$m run lat_${m}_$P 200 python tools/oshrun -np $P --timeout 180 python tools/latency_check.py
    done
done
exit 0
