#!/bin/bash
# Two bench.py processes on the box's one GPU at once (diagnostic for the
# one-GPU multi-rank rehearsal): each must print its line without a runner
# error.  Args: bench.py arguments.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py "$@" > gpurun_out/conc_a.log 2>&1 &
pa=$!
timeout -k 10 300 python bench.py "$@" > gpurun_out/conc_b.log 2>&1 &
pb=$!
wait $pa; ra=$?
wait $pb; rb=$?
echo "a rc=$ra b rc=$rb"
grep -h "Error\|^{" gpurun_out/conc_a.log gpurun_out/conc_b.log | cut -c1-200
