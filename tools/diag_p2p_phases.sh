#!/bin/bash
# p2p call latency at P PEs on one GPU, device-heap operands on the p2p executor (small path
# off), interleaved A/B of variants given as name=ENV1=v1,ENV2=v2 words in $VARIANTS
# (default: the stream-mode entry boundary, SHMEMX_P2P_ENTRY host vs device).
# SOSX_P2P_TRACE=$TRACE adds the per-phase host times to the .err files.
# Output: gpurun_out/diag_<tag>/P<P>_<name>_<round>.{txt,err}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-entry}
out=gpurun_out/diag_$tag
mkdir -p "$out"
export SHMEMX_TRANSPORT=p2p SHMEMX_DEVICE_HEAP_SIZE=256M SHMEMX_STAGE_BYTES=64M SHMEMX_DEVICE=0 SHMEMX_SMALL_DEVICE=0 SOSX_P2P_TRACE=${TRACE:-0} LAT_REPS=${LAT_REPS:-300}
P=${P:-2}
VARIANTS=${VARIANTS:-host=SHMEMX_P2P_ENTRY=host device=SHMEMX_P2P_ENTRY=device}
for k in ${ROUNDS:-1 2}; do
  for v in $VARIANTS; do
    name=${v%%=*}
    envs=${v#*=}
    timeout -k 10 200 env ${envs//,/ } python3 tools/oshrun -np $P --timeout 180 python3 tools/latency_check.py --legs dev --ring > "$out/P${P}_${name}_$k.txt" 2> "$out/P${P}_${name}_$k.err" || exit 1
  done
done
echo done
