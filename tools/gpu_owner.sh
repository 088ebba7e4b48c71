#!/bin/bash
# owner-apply pipelined runner: its bitwise tests, then the default bench
# with SKGE_PIPE_OWNER=0 / 1 interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -k "${TESTK:-bitwise}" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_own.log 2>&1; rc=$?
tail -3 gpurun_out/t_own.log; [ $rc -ne 0 ] && exit $rc
ENVS=${ENVS:-"SKGE_PIPE_OWNER=0 SKGE_PIPE_OWNER=1"} ROUNDS=${ROUNDS:-2} BENCH_ARGS="--steps 20 --warmup 3" bash tools/gpu_abenv.sh
