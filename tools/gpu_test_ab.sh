#!/bin/bash
# GPU tests, then bench lines for each configuration in $CONFIGS
# (entries "name:libvariant:bench args", libvariant "-" = current library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
fi
for cfg in ${CONFIGS:-cur:-:}; do
  name=${cfg%%:*}; rest=${cfg#*:}; v=${rest%%:*}; args=${rest#*:}; args=${args//,/ }
  if [ "$v" = "-" ]; then lib=""; else lib=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  SKGE_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu $args > gpurun_out/ab_$name.log 2>&1 || exit $?
  python -c "
import json; l=[x for x in open('gpurun_out/ab_$name.log') if x.startswith('{')][0]; j=json.loads(l)
print('$name', j['value'], j['ms_per_step'], j['detail']['kernels'], j['detail']['violations_per_pair'])"
done
