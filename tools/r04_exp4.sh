#!/bin/bash
# Round-4 experiment batch 4: split apply / scoring kernels at large batches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKGE_PIPE_SPLIT=1 TAG=r04g STEPS="tests:tests/test_gpu_device_loop.py" bash tools/gpu_run.sh || exit $?
AB="s0 SKGE_PIPE_SPLIT=0;s1 SKGE_PIPE_SPLIT=1;s0b SKGE_PIPE_SPLIT=0;s1b SKGE_PIPE_SPLIT=1" timeout -k 10 400 bash tools/ab_pipe.sh || exit $?
SKGE_PIPE_SPLIT=1 TAG=r04pt2s STEPS="tool:pipe_trace.py,--nb,2,--launch,2" bash tools/gpu_run.sh || exit $?
TAG=r04ht2 STEPS="tool:hole_trace.py" bash tools/gpu_run.sh || exit $?
SKGE_HPIPE_SPEC=1 TAG=r04hs STEPS="tests:hole" bash tools/gpu_run.sh || exit $?
BENCHARGS="--config 3" AB="h0 SKGE_HPIPE_SPEC=0;h1 SKGE_HPIPE_SPEC=1;h0b SKGE_HPIPE_SPEC=0;h1b SKGE_HPIPE_SPEC=1" timeout -k 10 500 bash tools/ab_pipe.sh || exit $?
SKGE_HPIPE_SPEC=1 TAG=r04ht3 STEPS="tool:hole_trace.py" bash tools/gpu_run.sh || exit $?
exit 0
