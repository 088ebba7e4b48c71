#!/bin/bash
# Round-4: upper bound of a d-exact RESCAL tiling at d = 200 (timing-only build:
# the edge GEMM column block and edge dW tiles skip their contraction).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCHARGS="--config 4" timeout -k 10 900 bash tools/ab_lib.sh nopad=SKGE_ABL_RS_NOPAD || exit $?
exit 0
