#!/bin/bash
# Round-4: HolE pair form, apply-role cap around the residency default (626 workgroups at nb = 100).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCHARGS="--config 3" AB="dflt SKGE_X=0;c520 SKGE_HPIPE_ACAP=520;c580 SKGE_HPIPE_ACAP=580;c680 SKGE_HPIPE_ACAP=680;c760 SKGE_HPIPE_ACAP=760;dflt2 SKGE_X=0" timeout -k 10 700 bash tools/ab_pipe.sh || exit $?
exit 0
