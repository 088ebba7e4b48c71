#!/bin/bash
# GPU test pass: the full -m gpu suite (one process), then the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 300 \
  --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
[ -n "${NOBENCH:-}" ] && exit 0
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | cut -c1-400
