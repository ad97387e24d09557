#!/bin/bash
# Run named GPU steps on the gpurun box, each under its own time limit.
# Usage: tools/gpu_steps.sh "name|seconds|command" ...
# A step that fails an assertion (exit 1/2/...) lets the next step run; a GPU fault,
# abort, segfault or time limit (124/134/137/139 or signal) ends the script there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
    name="${spec%%|*}"; rest="${spec#*|}"
    secs="${rest%%|*}"; cmd="${rest#*|}"
    echo "=== step $name (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
    rc=$?
    echo "=== step $name rc=$rc wall=$(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
    tail -n 5 "gpurun_out/$name.out" "gpurun_out/$name.err" | tail -n 12
    case $rc in
        124|134|137|139) echo "fatal rc=$rc in step $name: stopping"; exit $rc ;;
    esac
    if [ $rc -ge 128 ]; then echo "signal rc=$rc in step $name: stopping"; exit $rc; fi
done
exit 0
