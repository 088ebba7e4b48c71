#!/bin/bash
# Round-4 experiment batch 10: large batches, pipelined vs two-launch (dense entity apply or not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/large_batch_ab.py --nb 2 > gpurun_out/lb_nb2.log 2>&1 || { tail -5 gpurun_out/lb_nb2.log; exit 1; }
SKGE_APPLY_DENSE=1 timeout -k 10 300 python tools/large_batch_ab.py --nb 2 --runners two-launch > gpurun_out/lb_nb2_dense.log 2>&1 || { tail -5 gpurun_out/lb_nb2_dense.log; exit 1; }
timeout -k 10 300 python tools/large_batch_ab.py --nb 10 > gpurun_out/lb_nb10.log 2>&1 || exit 1
SKGE_APPLY_DENSE=1 timeout -k 10 300 python tools/large_batch_ab.py --nb 10 --runners two-launch > gpurun_out/lb_nb10_dense.log 2>&1 || exit 1
grep -h '^{' gpurun_out/lb_nb*.log
exit 0
