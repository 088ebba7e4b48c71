#!/bin/bash
# Round-4: HolE pair form, twiddle table written before the loop (old) vs after
# the first record and row loads are issued (new default); HolE tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r04tw STEPS="tests:hole" bash tools/gpu_run.sh || exit $?
BENCHARGS="--config 3" timeout -k 10 900 bash tools/ab_lib.sh twfirst=SKGE_HPIPE_TW_FIRST || exit $?
exit 0
