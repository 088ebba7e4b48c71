#!/bin/bash
# Round-4: TransE nb = 2, scoring-workgroup cap (each scoring wave loops over more positives).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB="dflt SKGE_X=0;b2k SKGE_PIPE_BCAP=2048;b4k SKGE_PIPE_BCAP=4096;b8k SKGE_PIPE_BCAP=8192;dflt2 SKGE_X=0" timeout -k 10 600 bash tools/ab_pipe.sh || exit $?
exit 0
