#!/bin/bash
# Round-4 measurement 6: bf16 GEMM numerics first (short), then the VGG-11 side-stream A/B
# (round 3 vs the restored overlap, on/off) and the GEMM / Llama A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_bf16_gpu.py > gpurun_out/gemm_tests.log 2>&1
grc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gemm_tests.log | tail -8; echo "gemm pytest rc=$grc"
# a failed numerics test does not stop the VGG A/B (independent code); a crash / time limit does
case $grc in 0|1) ;; *) exit $grc ;; esac
V=".ab/r3 .ab/r4d .ab/r4d:CS_OVERLAP_WGRAD=0"
bash scripts/ab_trees.sh 3 $V -- --steps 20 --warmup 5 > gpurun_out/ab4_20_5.log 2>&1 || exit $?
tail -3 gpurun_out/ab4_20_5.log
bash scripts/ab_trees.sh 2 $V -- --steps 100 --warmup 10 > gpurun_out/ab4_100_10.log 2>&1 || exit $?
tail -3 gpurun_out/ab4_100_10.log
[ $grc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/gemm_bench.py --rounds 3 --reps 5 > gpurun_out/gemm_bench.log 2>&1 || exit $?
cat gpurun_out/gemm_bench.log
