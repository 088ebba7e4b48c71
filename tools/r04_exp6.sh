#!/bin/bash
# Round-4 experiment batch 6: HolE pair form on by default -- tests, then the
# apply-role cap and dispatch order A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r04hq STEPS="tests:tests/test_gpu_runner_oracle.py" bash tools/gpu_run.sh || exit $?
BENCHARGS="--config 3" AB="dflt SKGE_X=0;c400 SKGE_HPIPE_ACAP=400;c900 SKGE_HPIPE_ACAP=900;c1300 SKGE_HPIPE_ACAP=1300;bfirst SKGE_HPIPE_AFIRST=0;dflt2 SKGE_X=0" timeout -k 10 600 bash tools/ab_pipe.sh || exit $?
exit 0
