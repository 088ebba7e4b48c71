#!/bin/bash
# Round-4: config 1 (d = 50 on 64-wide rows, SGD) with one apply wave per positive (A4) vs per slot.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCHARGS="--config 1" AB="s0 SKGE_PIPE_A4=0;a4 SKGE_PIPE_A4=1;s0b SKGE_PIPE_A4=0;a4b SKGE_PIPE_A4=1" timeout -k 10 500 bash tools/ab_pipe.sh || exit $?
exit 0
