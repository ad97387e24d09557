#!/bin/bash
# Full-size rehearsal of the driver's N > 1 bench on ONE GPU (all ranks share it; RCCL
# refuses that, so the job runs on the p2p transport in both signalling modes).
# Usage: tools/rehearse_n2.sh [N ...]   (default: 2)
# With 8 ranks on one GPU, run it as GPU_MAX_HW_QUEUES=1 tools/rehearse_n2.sh 8: with the
# runtime's default queues per process the device's hardware queues are oversubscribed
# and every call waits on queue time-slicing (~21 ms per call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for n in "${@:-2}"; do
    start=$(date +%s)
    timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
        --master-addr 127.0.0.1 --master-port $((29555 + n)) bench.py --gpus "$n" --steps 20 \
        --warmup 5 > "gpurun_out/n$n.out" 2> "gpurun_out/n$n.err"
    rc=$?
    echo "N=$n rc=$rc wall=$(( $(date +%s) - start ))s"
    tail -3 "gpurun_out/n$n.err"
    [ $rc -eq 0 ] || exit $rc
done
