#!/bin/bash
# full GPU check: all gpu tests, smoke, pipelined + two-launch bench lines, trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for v in pipe:auto f32:f32; do
  n=${v%%:*}; acc=${v#*:}
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --acc $acc > gpurun_out/b_$n.log 2>&1 || exit $?
  python3 -c "
import json;j=json.loads([l for l in open('gpurun_out/b_$n.log') if l.startswith('{')][0]);print('$n',j['value'],j['ms_per_step'],j['detail']['runner'],j['detail']['kernels'])"
done
timeout -k 10 300 python tools/pipe_trace.py ${TRACE_ARGS:-} > gpurun_out/trace.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/trace.log
