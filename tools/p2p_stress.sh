#!/bin/bash
# tools/p2p_stress.py under tools/oshrun: P PEs on this box's one GPU, p2p transport.
# Usage: tools/p2p_stress.sh P SIGNAL ITERS [ALG]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export SHMEMX_TRANSPORT=p2p SHMEMX_DEVICE_HEAP_SIZE=256M SHMEMX_STAGE_BYTES=64M SHMEMX_DEVICE=0
export PYTHONPATH=$PWD SHMEMX_P2P_SIGNAL=${2:-host}
[ "${1:-12}" -ge 8 ] && export GPU_MAX_HW_QUEUES=1
exec python3 tools/oshrun -np "${1:-12}" --timeout 280 python3 tools/p2p_stress.py --iters "${3:-100}" --alg "${4:-recdbl_gather}"
