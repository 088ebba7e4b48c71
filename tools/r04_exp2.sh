#!/bin/bash
# Round-4 experiment batch 2: RESCAL GEMM K split (parity + A/B), config 5
# kernel-trace evidence.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r04f STEPS="tests:padded tests:config1 tests:test_dp" bash tools/gpu_run.sh || exit $?
timeout -k 10 900 bash tools/ab_lib.sh occ7=SKGE_PIPE_WAVES_PER_EU=7 occ8=SKGE_PIPE_WAVES_PER_EU=8 || exit $?
SKGE_RS_GKS=2 TAG=r04e STEPS="tests:rescal" bash tools/gpu_run.sh || exit $?
BENCHARGS="--config 4" AB="g1 SKGE_RS_GKS=1;g2 SKGE_RS_GKS=2;g1b SKGE_RS_GKS=1;g2b SKGE_RS_GKS=2" timeout -k 10 500 bash tools/ab_pipe.sh || exit $?
TAG=r04s5 STEPS="stats:--config,5,--steps,2,--warmup,1,--no-cpu" bash tools/gpu_run.sh || exit $?
python3 tools/trace_by_grid.py gpurun_out/r04s5_stats1 > gpurun_out/r04s5_stats1/kernel_trace_by_grid.json || true
exit 0
