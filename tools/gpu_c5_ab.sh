#!/bin/bash
# config 5 (|E| = 50M, d = 512) with the current library and each
# build_abl/<variant>, same box; prints value and the two kernels' times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in cur ${VARIANTS:-}; do
  if [ $v = cur ]; then lib=""; else lib=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  SKGE_LIB_PATH=$lib timeout -k 10 500 python bench.py --config 5 --steps ${STEPS:-2} --warmup 1 --no-cpu \
    > gpurun_out/c5_$v.log 2>&1 || { tail -5 gpurun_out/c5_$v.log; exit 1; }
  python -c "
import json; l=[x for x in open('gpurun_out/c5_$v.log') if x.startswith('{')][0]; j=json.loads(l)
print('$v', j['value'], j['ms_per_step'], {k: (v['avg_us'], v['GB_s']) for k, v in j['detail']['kernels'].items()})"
done
