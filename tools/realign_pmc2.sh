set -u
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/realign_pmc2
mkdir -p $out
R=$(pwd)
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$out/fetch" -o fetch -- python3 tools/realign_ab.py --only 0,5 --rounds 1 --reps 2 --layouts mixed > $out/fetch.out 2> $out/fetch.err || exit 1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$out/write" -o write -- python3 tools/realign_ab.py --only 0,5 --rounds 1 --reps 2 --layouts mixed > $out/write.out 2> $out/write.err || exit 1
echo ok
