#!/bin/bash
# quick GPU iteration: GPU tests (stop on first failure) + one bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:---no-cpu} > gpurun_out/b_quick.log 2>&1 || exit $?
python - <<'PY'
import json
l=[x for x in open('gpurun_out/b_quick.log') if x.startswith('{')][0]; j=json.loads(l)
print(j['value'], j['ms_per_step'], j['roofline']['achieved'], j['detail']['kernels'], j['detail']['violations_per_pair'])
PY
