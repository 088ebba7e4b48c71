#!/bin/bash
# HolE A/B in one box: GPU tests of the HolE paths, then bench --config 3 with
# the current library and each build_abl/<variant> (tools/build_rev.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_hole.log 2>&1; rc=$?
  tail -5 gpurun_out/pytest_hole.log; [ $rc -ne 0 ] && exit $rc
fi
for v in cur ${VARIANTS:-base}; do
  if [ $v = cur ]; then lib=""; else lib=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  for c in ${CONFIGS:-3}; do
    SKGE_LIB_PATH=$lib timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 --no-cpu \
      ${BENCH_ARGS:-} > gpurun_out/hab_${v}_$c.log 2>&1 || exit $?
    python -c "
import json; l=[x for x in open('gpurun_out/hab_${v}_$c.log') if x.startswith('{')][0]; j=json.loads(l)
print('$v c$c', j['value'], j['ms_per_step'], j['detail'].get('kernels'))"
  done
done
