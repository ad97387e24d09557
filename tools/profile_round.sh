#!/bin/bash
# Collect this round's rocprof evidence on the GPU box into gpurun_out/prof_<tag>/ and
# the summaries into profiles/ (copy back + commit).  Usage: tools/profile_round.sh r1
# Kernel-trace stats and each PMC counter run in SEPARATE rocprofv3 passes.
set -u
tag=${1:-r1}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
run() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    echo "=== $name" >> "$out/steps.log"
    timeout -k 10 "$secs" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "=== $name rc=$rc" >> "$out/steps.log"
    case $rc in 0) ;; *) echo "step $name failed rc=$rc"; exit $rc ;; esac
}
R=$(pwd)
# 1. headline combine, kernel trace + stats
run combine_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/combine" -o combine -- python3 bench.py --no-pmc --no-cpu --no-host --no-adjacent --steps 50
# 2. PMC passes (one counter group per pass)
run combine_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$out/fetch" -o fetch -- python3 bench.py --child-pmc --steps 5 --warmup 1
run combine_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$out/write" -o write -- python3 bench.py --child-pmc --steps 5 --warmup 1
# 3. team fold kernel on 8 loopback PEs at the headline size
run loopback_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/loopback" -o loopback -- python3 tools/loopback_bench.py --P 8 --n 134217728 --alg ring
exit 0
