#!/bin/bash
# Round-4 measurement 5: bf16 matrix-core GEMM (gemm_bf16.hip) numerics + Llama-shape A/B vs
# hipBLASLt, then the working-tree measurements of r4_next.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_bf16_gpu.py > gpurun_out/gemm_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gemm_tests.log | tail -20; echo "gemm pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_bench.py --rounds 3 --reps 5 > gpurun_out/gemm_bench.log 2>&1 || exit $?
cat gpurun_out/gemm_bench.log
bash scripts/ab_trees.sh 2 .:CS_LM_GEMM=blas .:CS_LM_GEMM=native -- --model llama3-8b --steps 6 --warmup 3 \
  > gpurun_out/ab_llama_gemm.log 2>&1 || exit $?
tail -2 gpurun_out/ab_llama_gemm.log
if [ "${1:-}" = "next" ]; then bash scripts/r4_next.sh; fi
