#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base rs_noloadw rs_nomfma rs_noepi; do
  if [ $v = base ]; then LIBP=""; else LIBP=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  D=gpurun_out/prof_rs_$v; rm -rf $D; mkdir -p $D
  SKGE_LIB_PATH=$LIBP timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D -o run -- python3 tools/bench_models.py --models rescal > $D/log 2>&1 || exit $?
  echo "== $v"; f=$(find $D -name "*kernel_stats.csv" | head -1); cut -d, -f1,4 $f | grep rescal
done
