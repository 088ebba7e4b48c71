#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
T="tests/test_gpu_models.py -k rescal"
timeout -k 10 300 python -m pytest $T -q -p no:cacheprovider > gpurun_out/rs_mfma.log 2>&1
echo "mfma: $(tail -1 gpurun_out/rs_mfma.log)"; grep "elements off" gpurun_out/rs_mfma.log | head -5
SKGE_RESCAL_VALU=1 timeout -k 10 300 python -m pytest $T -q -p no:cacheprovider > gpurun_out/rs_valu.log 2>&1
echo "valu: $(tail -1 gpurun_out/rs_valu.log)"; grep "elements off" gpurun_out/rs_valu.log | head -5
