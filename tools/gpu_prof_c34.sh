#!/bin/bash
# rocprofv3 kernel stats of bench.py --config 3 (HolE) and --config 4 (RESCAL)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CONFIGS:-3 4}; do
  D=gpurun_out/prof_c$c
  rm -rf $D; mkdir -p $D
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D -o run -- \
    python3 bench.py --config $c --steps ${STEPS:-3} --warmup 1 --no-cpu > $D/bench.json 2> $D/log || exit $?
  f=$(find $D -name "*kernel_stats.csv" | head -1)
  cp $f $D/kernel_stats.csv
  echo "== config $c"; cat $D/bench.json | cut -c1-200
  cut -d, -f1-5 $D/kernel_stats.csv | head -14
done
