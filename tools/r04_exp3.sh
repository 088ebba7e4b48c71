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
SKGE_BENCH_BACKEND=gloo SKGE_BENCH_ONE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --large-nb 0 > gpurun_out/r04_dry2.log 2>&1
rc=$?; echo "== two-rank rehearsal rc=$rc"; grep '^{' gpurun_out/r04_dry2.log | cut -c1-3000; tail -5 gpurun_out/r04_dry2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TAG=r04pt2 STEPS="tool:pipe_trace.py,--nb,2,--launch,2" bash tools/gpu_run.sh || exit $?
exit 0
