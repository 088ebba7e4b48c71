#!/bin/bash
# RESCAL dW kernel timing ablations (variant builds from tools/ablate.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base nomfma noapply; do
  if [ $v = base ]; then L=""; else L=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  SKGE_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/wabl_$v -o run -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu > gpurun_out/wabl_$v.log 2>&1 || exit $?
  echo "== $v"; grep -h "k_rescal" $(find gpurun_out/wabl_$v -name "*kernel_stats.csv") | cut -d, -f1-4
done
