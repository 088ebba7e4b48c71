#!/bin/bash
# Round-4: per-batch entity count bound -- skewed-KG tests, device-loop tests,
# and the skewed KG at nb = 10 / 2 (bench detail lines).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r04sb STEPS="tests:tests/test_gpu_skew.py tests:tests/test_gpu_device_loop.py tests:tests/test_gpu_dp.py" bash tools/gpu_run.sh || exit $?
timeout -k 10 300 python bench.py --skew zipf --nb 10 --steps 10 --warmup 2 --no-cpu --no-roofline --large-nb 0 > gpurun_out/bench_zipf_nb10.log 2>&1 || { tail -5 gpurun_out/bench_zipf_nb10.log; exit 1; }
grep -h '^{' gpurun_out/bench_zipf_nb10.log | cut -c1-300
exit 0
