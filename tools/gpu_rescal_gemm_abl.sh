#!/bin/bash
# RESCAL GEMM (k_rescal_gemm) timing ablations: variant builds from tools/ablate.sh
# (build_abl/<v>: nomfma=SKGE_ABL_GEMM_NOMFMA, noload=SKGE_ABL_GEMM_NOLOAD, bare=both),
# each profiled on bench.py --config 4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base ${VARIANTS:-nomfma noload bare}; do
  if [ $v = base ]; then L=""; else L=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  SKGE_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/gabl_$v -o run -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu --large-nb 0 > gpurun_out/gabl_$v.log 2>&1 || exit $?
  echo "== $v"; grep -h "k_rescal" $(find gpurun_out/gabl_$v -name "*kernel_stats.csv") | cut -d, -f1-4
done
