#!/bin/bash
# Round-4 measurement 11: bf16 GEMM schedules — numerics (every schedule bitwise vs the 4-phase
# pipeline, all layouts / output modes / split-K) and the Llama-shape bench of schedules 0 / 1 / 2
# against hipBLASLt in one process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_bf16_gpu.py tests/test_gemm_sched_gpu.py > gpurun_out/gemm_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gemm_tests.log | tail -8; echo "gemm pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/gemm_bench.py --rounds 3 --reps 5 --sched-ab 1,2 > gpurun_out/gemm_bench.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/gemm_bench.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l) if l.startswith('{') else None
    d and print(d['shape'], d['product'], d['ours_tflops_med'], d['hipblaslt_tflops_med'], d['ours_vs_hipblaslt'], d.get('sched1_vs_hipblaslt'), d.get('sched2_vs_hipblaslt'))"
# same-box kernel traces of the round-2 tree and the working tree (where is round 2's remaining lead?)
R=$PWD
trace_tree() {
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d $R/gpurun_out/$2 -o run -- \
    python3 $R/$1/bench.py --steps 10 --warmup 5 > $R/gpurun_out/$2.log 2>&1) || return $?
  python3 scripts/prof_summary.py gpurun_out/$2 --steps 15 --top 45 > gpurun_out/${2}_kernels.txt 2>&1
  python3 scripts/step_timeline.py gpurun_out/$2 > gpurun_out/${2}_timeline.txt 2>&1
  tail -3 gpurun_out/${2}_timeline.txt
}
trace_tree .ab/r2 r2_trace && trace_tree . r4_trace
bash scripts/ab_trees.sh 2 .:CS_CONV_GEMM=blas .:CS_CONV_GEMM=auto -- --model resnet50 --dtype bf16 --steps 10 \
  --warmup 4 > gpurun_out/ab_resnet_gemm.log 2>&1 || exit $?
tail -2 gpurun_out/ab_resnet_gemm.log
