#!/bin/bash
# HolE FFT vs direct correlations on one box: the HolE GPU tests, then bench
# --config 3 with the FFT path (default) and SKGE_HOLE_DIRECT=1, then the
# per-wave trace of the FFT path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  -k "${PYTEST_K:-hole or HolE or parity or models}" > gpurun_out/pytest_fft.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_fft.log; [ $rc -ne 0 ] && exit $rc
for v in fft direct; do
  if [ $v = direct ]; then export SKGE_HOLE_DIRECT=1; else unset SKGE_HOLE_DIRECT; fi
  timeout -k 10 300 python bench.py --config 3 --steps 20 --warmup 3 --no-cpu > gpurun_out/fft_$v.log 2>&1 || exit $?
  python -c "
import json; l=[x for x in open('gpurun_out/fft_$v.log') if x.startswith('{')][0]; j=json.loads(l)
print('$v', j['value'], j['ms_per_step'], j['detail']['violations_per_pair'], j['detail']['large_batch'])"
done
unset SKGE_HOLE_DIRECT
timeout -k 10 300 python tools/hole_trace.py > gpurun_out/hole_trace.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/hole_trace.log | tail -19
