#!/bin/bash
# Round-4: HolE pair form at mid batch sizes (nb = 50, 20), forced on vs off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCHARGS="--config 3 --nb 50" AB="n50p0 SKGE_HPIPE_PAIR=0;n50p1 SKGE_HPIPE_PAIR=1" timeout -k 10 400 bash tools/ab_pipe.sh || exit $?
BENCHARGS="--config 3 --nb 20" AB="n20p0 SKGE_HPIPE_PAIR=0;n20p1 SKGE_HPIPE_PAIR=1" timeout -k 10 400 bash tools/ab_pipe.sh || exit $?
exit 0
