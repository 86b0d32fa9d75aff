#!/bin/bash
# Round-4 measurement 9: GEMM v2 (fragment reuse across phases) numerics + Llama-shape bench, then
# r4_next2.sh (warm-up ramp, probe projection with CTA footprints, extension A/Bs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
T="tests/test_gemm_bf16_gpu.py"
python3 -c "from cs744_pytorch_distributed_tutorial_amd.ops import native; assert hasattr(native.C(), 'gemm_bf16_sched')" \
  2>/dev/null && T="$T tests/test_gemm_sched_gpu.py"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  $T > gpurun_out/gemm_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gemm_tests.log | tail -8; echo "gemm pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_bench.py --rounds 3 --reps 5 --sched-ab > gpurun_out/gemm_bench.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/gemm_bench.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l) if l.startswith('{') else None
    d and print(d['shape'], d['product'], d['ours_tflops_med'], d['hipblaslt_tflops_med'], d['ours_vs_hipblaslt'], d.get('sched1_vs_hipblaslt'))"
bash scripts/r4_next2.sh
