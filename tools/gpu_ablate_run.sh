set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b_base.log 2>&1 || exit $?
for v in noratom noeatom; do
  SKGE_LIB_PATH=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b_$v.log 2>&1 || exit $?
done
for f in base noratom noeatom; do python -c "
import json,sys; l=[x for x in open('gpurun_out/b_$f.log') if x.startswith('{')][0]; j=json.loads(l); print('$f', j['value'], j['ms_per_step'], j['detail']['kernels'])"; done
