#!/bin/bash
# pipelined runner: device-loop tests, a bench line, a per-wave trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_device_loop.py -q -x -p no:cacheprovider > gpurun_out/pytest_pipe.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_pipe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b_pipe.log 2>&1 || exit $?
python3 -c "
import json;j=json.loads([l for l in open('gpurun_out/b_pipe.log') if l.startswith('{')][0]);print(j['value'],j['ms_per_step'],j['detail']['kernels'])"
timeout -k 10 300 python tools/pipe_trace.py ${TRACE_ARGS:-} > gpurun_out/trace.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/trace.log
