#!/bin/bash
# One-GPU N=8 bench latency diagnosis: the bench at 1Mi elements under torchrun, p2p only,
# with the HIP runtime's default number of hardware queues per process and with one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export PYTHONPATH=$(pwd) SHMEMX_DEVICE=0
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > gpurun_out/$name.out 2> gpurun_out/$name.err; local rc=$?; echo "rc=$rc"; grep -o '"transports": {[^}]*}[^}]*}[^}]*}' gpurun_out/$name.out; grep -h "trace" gpurun_out/$name.err | tail -3; [ $rc -eq 0 ] || exit $rc; }
B="bench.py --gpus 8 --steps 10 --warmup 2 --nreduce 1048576 --no-team-sweep --no-host --no-adjacent --no-cpu"
SOSX_P2P_TRACE=10 run bench8_q1 300 env GPU_MAX_HW_QUEUES=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29601 $B
SOSX_P2P_TRACE=10 run bench4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29602 ${B/--gpus 8/--gpus 4}
