#!/bin/bash
# rocprofv3 kernel stats of the HolE config-3 bench under both device runners
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for r in ${RUNNERS:-pairs hole_pipe}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_$r -o run --output-format csv -- python3 bench.py --config 3 --no-cpu --steps 5 --warmup 1 --runner $r > gpurun_out/prof_c3_$r.log 2>&1 || { tail -5 gpurun_out/prof_c3_$r.log; exit 1; }
  f=$(find gpurun_out/prof_c3_$r -name "*kernel_stats.csv" | head -1)
  echo "== $r"; cut -d, -f1-4 "$f" | head -8
done
