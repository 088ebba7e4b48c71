#!/bin/bash
# Round-4 experiment batch 7: per-wave traces of the HolE pair form and the one-wave form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r04hr STEPS="tests:hole" bash tools/gpu_run.sh || exit $?
TAG=r04htp STEPS="tool:hole_trace.py" bash tools/gpu_run.sh || exit $?
SKGE_HPIPE_PAIR=0 TAG=r04ht1 STEPS="tool:hole_trace.py" bash tools/gpu_run.sh || exit $?
exit 0
