#!/bin/bash
# Round-4 measurement 18: PMC passes (counter collection only, no trace domains) — the bf16 GEMM vs
# hipBLASLt at the Llama w1/w3 shape, and the VGG-11 step's kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
CNT="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $CNT --output-format csv -d $R/gpurun_out/gemm_pmc -o run -- \
  python3 $R/scripts/gemm_bench.py --rounds 1 --reps 1 --shapes w1/w3 > $R/gpurun_out/gemm_pmc.log 2>&1)
rc=$?; echo "gemm pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py gpurun_out/gemm_pmc > gpurun_out/gemm_pmc_summary.txt 2>&1; head -12 gpurun_out/gemm_pmc_summary.txt
bash scripts/gpu.sh pmc vgg_pmc "$CNT" --steps 3 --warmup 2
