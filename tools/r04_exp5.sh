#!/bin/bash
# Round-4 experiment batch 5: HolE pair form (two waves per positive).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKGE_HPIPE_PAIR=1 TAG=r04hp STEPS="tests:hole" bash tools/gpu_run.sh || exit $?
BENCHARGS="--config 3" AB="h0 SKGE_HPIPE_PAIR=0;h1 SKGE_HPIPE_PAIR=1;h0b SKGE_HPIPE_PAIR=0;h1b SKGE_HPIPE_PAIR=1" timeout -k 10 500 bash tools/ab_pipe.sh || exit $?
exit 0
