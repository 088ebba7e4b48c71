#!/bin/bash
# Round-4 check: bench.py --gpus 2 end to end on a one-GPU box (both ranks on
# GPU 0 over gloo: the launcher, the rank setup, the max-over-ranks timing and
# the replica line; RCCL itself needs two GPUs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKGE_BENCH_ONE_GPU=1 SKGE_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_g2_onegpu.log 2>&1 || { tail -20 gpurun_out/bench_g2_onegpu.log; exit 1; }
grep '^{' gpurun_out/bench_g2_onegpu.log
exit 0
