#!/bin/bash
# rocprofv3 evidence for the round: the default bench line, kernel-trace stats
# of the same bench command, then FETCH_SIZE and WRITE_SIZE in separate --pmc
# passes (never combined with other trace domains); summarised per kernel (and
# per launch geometry) into gpurun_out/prof_$TAG/pmc.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=${TAG:-r01}
ARGS=${ARGS:---steps 20 --warmup 3 --no-cpu}   # the default bench workload (no CPU leg)
export TMPDIR=/tmp
D=gpurun_out/prof_$TAG
mkdir -p $D
timeout -k 10 300 python3 bench.py $ARGS > $D/bench.log 2>&1 || { tail $D/bench.log; exit 1; }
grep '^{' $D/bench.log > $D/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D/stats -o run -- python3 bench.py $ARGS > $D/stats.log 2>&1 || exit $?
grep '^{' $D/stats.log > $D/bench_under_rocprof.json
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d $D/fetch -o run -- python3 bench.py $ARGS > $D/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d $D/write -o run -- python3 bench.py $ARGS > $D/write.log 2>&1 || exit $?
python3 tools/pmc_summary.py $D > $D/pmc.json && cat $D/bench.json && python3 -c "
import json; d=json.load(open('$D/pmc.json'))
for k,v in d.items():
    if 'pipe' in k or 'roofline' in k: print(k, json.dumps(v)[:600])"
