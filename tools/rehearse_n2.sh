#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
start=$(date +%s)
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/n2.out 2> gpurun_out/n2.err
rc=$?
echo "rc=$rc wall=$(( $(date +%s) - start ))s"
tail -3 gpurun_out/n2.err
exit $rc
