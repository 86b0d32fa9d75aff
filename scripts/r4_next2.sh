#!/bin/bash
# Round-4 measurement 8: extension A/Bs on the native GEMM (r4_ext.sh), then the 20/5 warm-up ramp
# and the one-GPU probe projection of N = 2/4/8 (xGMI-model collectives, CS_COMM_CTAS sweep).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_ramp.py --warmup 5 --window 20 --windows 10 > gpurun_out/ramp.log 2>&1 || exit $?
tail -4 gpurun_out/ramp.log
timeout -k 10 500 python -u scripts/dp_projection.py --steps 40 --warmup 10 --gbps 150,300 > gpurun_out/dp_projection.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/dp_projection.log
bash scripts/r4_ext.sh
