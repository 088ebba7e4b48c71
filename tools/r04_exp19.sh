#!/bin/bash
# Round-4 final check: the config 1 / 3 / 4 bench lines with the final bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 1 3 4; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 > gpurun_out/fin_c$c.log 2>&1 || { tail -5 gpurun_out/fin_c$c.log; exit 1; }
  grep -h '^{' gpurun_out/fin_c$c.log | cut -c1-200
done
exit 0
