#!/bin/bash
# the headline bench line and the config-5 line, logs under gpurun_out/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/b_default.log 2>&1 || { tail -5 gpurun_out/b_default.log; exit 1; }
grep "^{" gpurun_out/b_default.log
timeout -k 10 900 python bench.py --config 5 --steps 2 --warmup 1 > gpurun_out/c5_full.log 2>&1 || { tail -5 gpurun_out/c5_full.log; exit 1; }
grep "^{" gpurun_out/c5_full.log
