#!/bin/bash
# Sharded config-5 bench on one GPU (G = 1: exchanges are identities) at a
# reduced and at the full size, plus the replica runner for comparison.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config 5 --shard --c5-scale ${SCALE:-0.25} --steps 2 --warmup 1 > gpurun_out/shard_bench_small.log 2>&1 || { tail -20 gpurun_out/shard_bench_small.log; exit 1; }
grep '^{' gpurun_out/shard_bench_small.log
if [ "${FULL:-0}" = 1 ]; then
timeout -k 10 900 python -u bench.py --config 5 --shard --steps 2 --warmup 1 > gpurun_out/shard_bench_full.log 2>&1 || { tail -20 gpurun_out/shard_bench_full.log; exit 1; }
grep '^{' gpurun_out/shard_bench_full.log
fi
