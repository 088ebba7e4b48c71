#!/bin/bash
# Copy one round's evidence (tools/evidence.sh outputs under gpurun_out/) into
# profiles/$ROUND/ under the names the bench lines and DESIGN cite:
# pmc[_c<k>].json, kernel_trace_by_grid[_c<k>].json, kernel_stats[_c<k>].csv,
# bench_default.json / bench_c<k>.json.  Usage: ROUND=r06 CONFIGS="2 1" tools/collect_evidence.sh
set -u
cd "$(dirname "$0")/.."
R=${ROUND:-r06}
mkdir -p profiles/$R
for c in ${CONFIGS:-2 1 3 4 5}; do
  suf=$([ "$c" = 2 ] && echo "" || echo "_c$c")
  D=gpurun_out/${R}p${c}_pmc1
  [ -f $D/pmc.json ] && cp $D/pmc.json profiles/$R/pmc$suf.json
  [ -f $D/kernel_trace_by_grid.json ] && cp $D/kernel_trace_by_grid.json profiles/$R/kernel_trace_by_grid$suf.json
  [ -f $D/stats/run_kernel_stats.csv ] && cp $D/stats/run_kernel_stats.csv profiles/$R/kernel_stats$suf.csv
  [ -f $D/kernel_trace_epochs.json ] && cp $D/kernel_trace_epochs.json profiles/$R/kernel_trace_epochs$suf.json
  b=gpurun_out/${R}p${c}_bench1.json
  [ -s $b ] && cp $b profiles/$R/$([ "$c" = 2 ] && echo bench_default.json || echo bench_c$c.json)
done
ls profiles/$R
