#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault / abort / timeout stops the
# script (plain test failures, rc 1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r01}
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  return $rc
}
step pytest_gpu 1200 python -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout=400
rc=$?; [ $rc -gt 1 ] && exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py --steps ${STEPS:-10} --warmup 2 || exit $?
cat gpurun_out/bench.log | grep '^{' > gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
cd - > /dev/null
step rocprof 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu || exit $?
find gpurun_out/prof_$TAG -name "*stats*" | head
