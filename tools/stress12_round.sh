#!/bin/bash
# The 12-PE stress of DESIGN.md section 5.4 on the current library: tools/p2p_stress.py --release
# under tools/oshrun -np 12 (p2p, host signalling, GPU_MAX_HW_QUEUES=1, 800 iterations), $RUNS runs.
# Output: gpurun_out/stress12/run<k>.{out,err}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/stress12
TAG=${TAG:-run}
export SHMEMX_TRANSPORT=p2p SHMEMX_P2P_SIGNAL=host GPU_MAX_HW_QUEUES=1
for k in $(seq 1 ${RUNS:-2}); do
  timeout -k 10 400 python3 tools/oshrun -np 12 --timeout 380 python3 tools/p2p_stress.py --release --iters 800 > gpurun_out/stress12/${TAG}$k.out 2> gpurun_out/stress12/${TAG}$k.err
  rc=$?
  echo "run $k rc=$rc clean PEs: $(grep -o 'checks OK' gpurun_out/stress12/${TAG}$k.out | wc -l)"
  [ $rc -eq 0 ] || exit $rc
done
