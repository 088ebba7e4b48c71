#!/bin/bash
# Round-4 experiment batch 9: HolE pair form, relation row on wave 0 vs wave 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKGE_HPIPE_PAIR_R1=1 TAG=r04hs1 STEPS="tests:hole" bash tools/gpu_run.sh || exit $?
BENCHARGS="--config 3" AB="r0 SKGE_HPIPE_PAIR_R1=0;r1 SKGE_HPIPE_PAIR_R1=1;r0b SKGE_HPIPE_PAIR_R1=0;r1b SKGE_HPIPE_PAIR_R1=1" timeout -k 10 500 bash tools/ab_pipe.sh || exit $?
exit 0
