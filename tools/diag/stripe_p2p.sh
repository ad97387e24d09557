#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
B="bench.py --gpus 2 --steps 5 --warmup 2 --no-team-sweep --no-adjacent --no-cpu"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 $B > gpurun_out/s0.out 2> gpurun_out/s0.err || exit 1
SHMEMX_HOST_STRIPE_BYTES=262144 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 $B > gpurun_out/s1.out 2> gpurun_out/s1.err || exit 1
SHMEMX_HOST_STRIPE_BYTES=1048576 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 $B > gpurun_out/s2.out 2> gpurun_out/s2.err || exit 1
for f in s0 s1 s2; do grep -o '"host_resident": {[^}]*}[^}]*}[^}]*}' gpurun_out/$f.out; done
