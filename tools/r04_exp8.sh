#!/bin/bash
# Round-4 experiment batch 8: HolE pair form at 5 waves per SIMD (compile-time variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCHARGS="--config 3" timeout -k 10 900 bash tools/ab_lib.sh occ5=SKGE_HPIPE_OCC=5 || exit $?
exit 0
