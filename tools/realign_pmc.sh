#!/bin/bash
# HBM traffic of the realigning fold and prefix: the 8-input fold and
# SUM prefix over 16Mi fp32 per input with every input at its own 16-B offset ("mixed":
# k_fold_realign_np / k_prefix_realign_np) beside the congruent layout (k_fold / k_prefix),
# tools/misaligned_probe.py.  Kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes.  Output: gpurun_out/realign_pmc/.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/realign_pmc${REALIGN_TAG:-}
mkdir -p "$out"
R=$(pwd)
run() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    echo "=== $name $(date +%T)"
    timeout -k 10 "$secs" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "=== $name rc=$rc $(date +%T)"
    [ $rc -eq 0 ] || { tail -20 "$out/$name.err"; exit $rc; }
}
run warm 300 python3 -c "import torch; torch.cuda.init()"
for k in fold prefix; do
    run ${k}_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/${k}_stats" -o stats -- python3 tools/misaligned_probe.py --$k --only congruent,mixed --reps 10
    run ${k}_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$out/${k}_fetch" -o fetch -- python3 tools/misaligned_probe.py --$k --only congruent,mixed --reps 3
    run ${k}_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$out/${k}_write" -o write -- python3 tools/misaligned_probe.py --$k --only congruent,mixed --reps 3
done
exit 0
