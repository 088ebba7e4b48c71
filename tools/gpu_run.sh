#!/bin/bash
# One parameterised GPU-box driver (replaces the round-1/2 one-off gpu_*.sh
# scripts).  Steps, chosen by the STEPS env (space separated, run in order;
# each under its own time limit; a fault / abort / timeout stops the script,
# plain test failures (rc 1) do not):
#   tests[:<pytest -k expr or node ids>]  GPU tests (PYTEST_ARGS adds flags)
#   smoke                                 __graft_entry__.smoke()
#   bench[:<bench.py args>]               one bench line -> gpurun_out/<TAG>_bench*.json
#   stats[:<bench.py args>]               rocprofv3 --kernel-trace --stats of a bench command
#   pmc[:<bench.py args>]                 kernel-trace stats, then FETCH_SIZE and WRITE_SIZE passes
#                                         (separate runs) + tools/pmc_summary.py
#   pmcx[:<bench.py args>]                one --pmc pass of the counters in $PMCX + tools/pmc_counters.py
#   tool:<script>[,<args>]                python tools/<script> (or bash for .sh) under a time limit
# Arguments after ':' use ',' for spaces (e.g. bench:--config,3,--steps,5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
export TMPDIR=/tmp
n=0
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -${TAILN:-4} "gpurun_out/$name.log"
  return $rc
}
for st in ${STEPS:-tests smoke bench}; do
  n=$((n + 1))
  kind=${st%%:*}
  arg=""; [ "$kind" != "$st" ] && arg=$(echo "${st#*:}" | tr ',' ' ')
  case $kind in
    tests)
      if [ -n "$arg" ] && [[ "$arg" != *"::"* ]] && [[ "$arg" != tests/* ]]; then
        run ${TAG}_tests$n ${TTEST:-900} python -u -m pytest tests -m gpu -q -rf -x -p no:cacheprovider \
          --timeout ${TIMEOUT1:-300} --timeout-method thread -k "$arg" ${PYTEST_ARGS:-}
      else
        run ${TAG}_tests$n ${TTEST:-900} python -u -m pytest ${arg:-tests} -m gpu -q -rf -p no:cacheprovider \
          --timeout ${TIMEOUT1:-300} --timeout-method thread ${PYTEST_ARGS:-}
      fi
      rc=$?; if [ $rc -gt 1 ]; then exit $rc; fi ;;
    smoke)
      run ${TAG}_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)
      run ${TAG}_bench$n ${TBENCH:-600} python bench.py ${arg:---steps 20 --warmup 3} || exit $?
      grep '^{' gpurun_out/${TAG}_bench$n.log > gpurun_out/${TAG}_bench$n.json ;;
    stats)
      D=gpurun_out/${TAG}_stats$n
      run ${TAG}_stats$n 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D -o run \
        -- python3 bench.py ${arg:---steps 20 --warmup 3 --no-cpu} || exit $?
      grep '^{' gpurun_out/${TAG}_stats$n.log > $D/bench_under_rocprof.json ;;
    pmc)
      D=gpurun_out/${TAG}_pmc$n
      run ${TAG}_pmcs$n 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D/stats -o run \
        -- python3 bench.py ${arg:---steps 20 --warmup 3 --no-cpu} || exit $?
      grep '^{' gpurun_out/${TAG}_pmcs$n.log > $D/bench_under_rocprof.json
      run ${TAG}_pmcf$n 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv \
        -d $D/fetch -o run -- python3 bench.py ${arg:---steps 20 --warmup 3 --no-cpu} || exit $?
      run ${TAG}_pmcw$n 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv \
        -d $D/write -o run -- python3 bench.py ${arg:---steps 20 --warmup 3 --no-cpu} || exit $?
      python3 tools/pmc_summary.py $D > $D/pmc.json && echo "pmc summary: $D/pmc.json" ;;
    pmcx)   # one --pmc pass of the counters in $PMCX (space separated) over a bench command
      D=gpurun_out/${TAG}_pmcx$n
      run ${TAG}_pmcx$n 300 rocprofv3 --pmc ${PMCX:-SQ_WAVES SQ_WAVE_CYCLES} --kernel-trace -T \
        --output-format csv -d $D -o run -- python3 bench.py ${arg:---steps 5 --warmup 2 --no-cpu} || exit $?
      python3 tools/pmc_counters.py $D > $D/pmc_counters.json && echo "pmc counters: $D/pmc_counters.json" ;;
    tool)   # tool:<script under tools/>,<args>  (python scripts and .sh drivers)
      set -- $arg
      scr=$1; shift
      case $scr in
        *.sh) run ${TAG}_tool$n ${TTOOL:-600} bash tools/$scr "$@" || exit $? ;;
        *) run ${TAG}_tool$n ${TTOOL:-600} python -u tools/$scr "$@" || exit $? ;;
      esac ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
exit 0
