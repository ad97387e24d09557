set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/res
timeout -k 10 900 python -u -m pytest tests/test_gpu_multipe.py tests/test_gpu_team.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -k "resident or reduce_local_small" > gpurun_out/res/tests.log 2>&1 || { tail -30 gpurun_out/res/tests.log; exit 1; }
tail -2 gpurun_out/res/tests.log
export SHMEMX_TRANSPORT=p2p SHMEMX_DEVICE_HEAP_SIZE=256M SHMEMX_STAGE_BYTES=64M SHMEMX_DEVICE=0 LAT_REPS=500
# (device-heap operands: the small path up to SHMEMX_SMALL_DEVICE = 128 KiB per team)
for P in 2 4; do for k in 1 2; do for r in 0 1; do
  SHMEMX_SMALL_RESIDENT=$r timeout -k 10 200 python3 tools/oshrun -np $P --timeout 180 python3 tools/latency_check.py --legs ${LEGS:-host,dev} > gpurun_out/res/P${P}_r${r}_$k.txt 2> gpurun_out/res/P${P}_r${r}_$k.err || exit 1
done; done; done
echo done
