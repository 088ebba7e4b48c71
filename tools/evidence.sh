#!/bin/bash
# Evidence pass (per round: ROUND=r05 ...): the bench lines of every config plus their rocprofv3
# kernel-trace stats and FETCH_SIZE / WRITE_SIZE passes (gpu_run.sh `pmc`),
# summarised per kernel and grid (tools/pmc_summary.py, trace_by_grid.py).
# CONFIGS (default "2 1 3 4 5") selects; outputs under gpurun_out/${ROUND}p_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CONFIGS:-2 1 3 4 5}; do
  case $c in
    5) args="--config,5,--steps,2,--warmup,1" ;;
    *) args="--config,$c,--steps,20,--warmup,3" ;;
  esac
  TAG=${ROUND:-r05}p$c TBENCH=900 STEPS="bench:$args pmc:$args,--no-cpu" bash tools/gpu_run.sh || exit $?
  python3 tools/trace_by_grid.py gpurun_out/${ROUND:-r05}p${c}_pmc2/stats > gpurun_out/${ROUND:-r05}p${c}_pmc2/kernel_trace_by_grid.json || true
done
exit 0
