#!/bin/bash
# Round-4: skewed-KG GPU tests, then the config 2 / 3 bench lines on the Zipf KG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r04sk STEPS="tests:tests/test_gpu_skew.py" bash tools/gpu_run.sh || exit $?
exit 0
timeout -k 10 300 python bench.py --skew zipf --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_zipf_c2.log 2>&1 || { tail -5 gpurun_out/bench_zipf_c2.log; exit 1; }
timeout -k 10 300 python bench.py --skew zipf --config 3 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_zipf_c3.log 2>&1 || { tail -5 gpurun_out/bench_zipf_c3.log; exit 1; }
grep -h '^{' gpurun_out/bench_zipf_c2.log gpurun_out/bench_zipf_c3.log | cut -c1-400
exit 0
