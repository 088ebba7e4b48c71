#!/bin/bash
# Round-4 experiment batch (one GPU call): correctness of the A4 apply, A/Bs,
# the HolE SQ counter passes and the counter list.  Each step has its own time
# limit; a fault / timeout ends the script (gpu_run.sh semantics).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > gpurun_out/r04_counters.txt 2>&1 || true
SKGE_PIPE_A4=1 TAG=r04c STEPS="tests:tests/test_gpu_device_loop.py tests:tests/test_gpu_runner_oracle.py tests:tests/test_gpu_deterministic.py" bash tools/gpu_run.sh || exit $?
AB="base SKGE_PIPE_A4=0;a4 SKGE_PIPE_A4=1;base2 SKGE_PIPE_A4=0;a4b SKGE_PIPE_A4=1" timeout -k 10 400 bash tools/ab_pipe.sh || exit $?
SKGE_PIPE_A4=1 TAG=r04t4 STEPS="tool:pipe_trace.py" bash tools/gpu_run.sh || exit $?
BENCHARGS="--config 1" AB="c1p4 SKGE_PIPE_PAD_TO=4;c1p32 SKGE_PIPE_PAD_TO=32;c1p4a4 SKGE_PIPE_PAD_TO=4 SKGE_PIPE_A4=1;c1p32a4 SKGE_PIPE_PAD_TO=32 SKGE_PIPE_A4=1" timeout -k 10 400 bash tools/ab_pipe.sh || exit $?
TAG=r04d STEPS="tool:diag_pad_runners.py" bash tools/gpu_run.sh || exit $?
PMCX="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" TAG=r04h STEPS="pmcx:--config,3,--steps,3,--warmup,1,--no-cpu,--large-nb,0" bash tools/gpu_run.sh || exit $?
PMCX="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM" TAG=r04h2 STEPS="pmcx:--config,3,--steps,3,--warmup,1,--no-cpu,--large-nb,0" bash tools/gpu_run.sh || exit $?
exit 0
