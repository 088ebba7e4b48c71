set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base nocorr noatom; do
  if [ $v = base ]; then L=""; else L=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  SKGE_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/abl_$v -o run -- python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu > gpurun_out/abl_$v.log 2>&1 || exit $?
  echo "== $v"; grep -h "k_hole_pos\|k_apply" $(find gpurun_out/abl_$v -name "*kernel_stats.csv") | cut -d, -f1-4
done
