#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_models.py ${MODEL_ARGS:-} > gpurun_out/models.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/models.log | tail -5; exit $rc
