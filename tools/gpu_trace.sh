#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python tools/pipe_trace.py ${TRACE_ARGS:-} > gpurun_out/trace.log 2>&1; rc=$?
cat gpurun_out/trace.log | grep -v amdgpu.ids; exit $rc
