#!/bin/bash
# Round-4 experiment batch 3: TransE scoring-first dispatch A/B, the HolE
# per-wave trace, config 5 with per-kernel events over the timed epochs (+ its
# kernel-trace pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB="afirst SKGE_PIPE_AFIRST=1;bfirst SKGE_PIPE_AFIRST=0;afirst2 SKGE_PIPE_AFIRST=1;bfirst2 SKGE_PIPE_AFIRST=0" timeout -k 10 400 bash tools/ab_pipe.sh || exit $?
TAG=r04ht STEPS="tool:hole_trace.py" bash tools/gpu_run.sh || exit $?
TAG=r04s5b STEPS="stats:--config,5,--steps,2,--warmup,1,--no-cpu" bash tools/gpu_run.sh || exit $?
python3 tools/trace_by_grid.py gpurun_out/r04s5b_stats1 > gpurun_out/r04s5b_stats1/kernel_trace_by_grid.json || true
exit 0
