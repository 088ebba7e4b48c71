#!/bin/bash
# A/B in one box: microbenchmarks + bench with the current and the `prev` library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench > gpurun_out/ubench.log 2>&1; rc=$?; cat gpurun_out/ubench.log; [ $rc -ne 0 ] && exit $rc
for v in cur ${VARIANTS:-prev}; do
  if [ $v = cur ]; then lib=""; else lib=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  SKGE_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_$v.log 2>&1 || exit $?
  python -c "
import json; l=[x for x in open('gpurun_out/ab_$v.log') if x.startswith('{')][0]; j=json.loads(l)
print('$v', j['value'], j['ms_per_step'], j['detail']['kernels'])"
done
