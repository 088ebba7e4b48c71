#!/bin/bash
# Round-4: TransE large batches, two positives per scoring wave (SKGE_PIPE_P2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKGE_PIPE_P2=1 TAG=r04p2t STEPS="tests:tests/test_gpu_device_loop.py tests:tests/test_gpu_skew.py" bash tools/gpu_run.sh || exit $?
AB="q0 SKGE_PIPE_P2=0;q1 SKGE_PIPE_P2=1;q0b SKGE_PIPE_P2=0;q1b SKGE_PIPE_P2=1" timeout -k 10 500 bash tools/ab_pipe.sh || exit $?
exit 0
