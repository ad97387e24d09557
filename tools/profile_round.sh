#!/bin/bash
# Collect this round's rocprof evidence on the GPU box into gpurun_out/prof_<tag>/ (copy
# the summaries into profiles/ and commit).  Usage: tools/profile_round.sh r3
# Kernel-trace stats and each PMC counter run in SEPARATE rocprofv3 passes; every step
# has its own time limit and the script stops at the first failing step.
set -u
tag=${1:-r3}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
run() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    echo "=== $name $(date +%T)" | tee -a "$out/steps.log"
    timeout -k 10 "$secs" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "=== $name rc=$rc $(date +%T)" | tee -a "$out/steps.log"
    case $rc in 0) ;; *) echo "step $name failed rc=$rc"; tail -20 "$out/$name.err"; exit $rc ;; esac
}
R=$(pwd)
# 1. the driver's default N=1 line (runs its own PMC passes; raw CSVs kept)
run bench_n1 600 python3 bench.py --pmc-save "$R/$out/bench_pmc"
# 2. kernel trace + stats of the measured kernels only (headline combine, fold, prefix)
run kernel_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/stats" -o stats -- python3 bench.py --no-pmc --no-cpu --no-host --no-curve --steps 50
# 3. the fold inside the 8-PE loopback ring (plan-placed scratch slots): stats + PMC
run loopback_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/loopback" -o loopback -- python3 tools/loopback_bench.py --P 8 --n 134217728 --alg ring
run loopback_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$out/loopback_fetch" -o fetch -- python3 tools/loopback_bench.py --P 8 --n 134217728 --alg ring --iters 2
run loopback_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$out/loopback_write" -o write -- python3 tools/loopback_bench.py --P 8 --n 134217728 --alg ring --iters 2
exit 0
