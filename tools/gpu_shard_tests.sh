set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/shard_tests.log 2>&1; rc=$?
tail -30 gpurun_out/shard_tests.log; exit $rc
