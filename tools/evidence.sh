#!/bin/bash
# Evidence pass of a round (ROUND=r06 CONFIGS="2 1 3 4 5"): per config the
# rocprofv3 kernel-trace stats and FETCH_SIZE / WRITE_SIZE passes of the bench
# command (gpu_run.sh `pmc`), summarised per kernel and grid
# (tools/pmc_summary.py, trace_by_grid.py; config 5 also per epoch,
# tools/pmc_epochs.py / trace_epochs.py), installed as
# profiles/$ROUND/pmc[_c<k>].json BEFORE the config's bench line runs, so the
# line quotes this round's traffic (bench.PMC_ROUND).  Outputs under
# gpurun_out/${ROUND}p<k>_*; copy the summaries into profiles/$ROUND/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out "profiles/${ROUND:-r06}"
export TMPDIR=/tmp
R=${ROUND:-r06}
for c in ${CONFIGS:-2 1 3 4 5}; do
  case $c in
    5) args="--config,5,--steps,2,--warmup,1" ;;
    *) args="--config,$c,--steps,20,--warmup,3" ;;
  esac
  D=gpurun_out/${R}p${c}_pmc1
  TAG=${R}p$c TBENCH=900 STEPS="pmc:$args,--no-cpu" bash tools/gpu_run.sh || exit $?
  suf=$([ "$c" = 2 ] && echo "" || echo "_c$c")
  cp $D/pmc.json profiles/$R/pmc$suf.json
  python3 tools/trace_by_grid.py $D/stats > $D/kernel_trace_by_grid.json || true
  if [ "$c" = 5 ]; then   # the two-launch runner: nb launches of each batch kernel per epoch
    # full-batch launches per epoch: nb = T // B batches of T // nb positives,
    # the remainder a ragged batch (and, pipelined, the flush) at other grids
    nb=$(python3 -c "T = 100_000_000; bs = T // (T // 131072); print(T // bs)")
    python3 tools/pmc_epochs.py $D $nb > profiles/$R/pmc_c5_epochs.json || true
    python3 tools/trace_epochs.py $D/stats $nb > $D/kernel_trace_epochs.json || true
  fi
  TAG=${R}p$c TBENCH=900 STEPS="bench:$args" bash tools/gpu_run.sh || exit $?
done
exit 0
