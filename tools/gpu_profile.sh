#!/bin/bash
# rocprofv3 evidence for the round: kernel-trace stats of bench.py, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (never combined with other
# trace domains); summarised per kernel into gpurun_out/prof_$TAG/pmc.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=${TAG:-r01}
export TMPDIR=/tmp
D=gpurun_out/prof_$TAG
mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D/stats -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $D/stats.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d $D/fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $D/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d $D/write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $D/write.log 2>&1 || exit $?
python3 tools/pmc_summary.py $D > $D/pmc.json && cat $D/pmc.json
