#!/bin/bash
# per-kernel stats of tools/bench_models.py (MODELS env: comma list)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
D=gpurun_out/prof_models
rm -rf $D; mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D -o run -- python3 tools/bench_models.py --models ${MODELS:-rescal} > $D/log 2>&1 || exit $?
f=$(find $D -name "*kernel_stats.csv" | head -1)
cut -d, -f1-5 $f | head -20
