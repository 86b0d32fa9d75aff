# texture-address / L1 pressure of the conv GEMMs: is the GEMM bound by operand fetch?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
# counter collection serialises every dispatch: a kernel stream-link wait on the side stream would
# spin (until its 10 s timeout) waiting for a signal that cannot run -> profile the serial backward
export CS_OVERLAP_WGRAD=0
R=$GRAFT_REPO_ROOT
P1="TA_BUSY_avr GRBM_GUI_ACTIVE"
P2="TA_ADDR_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
P3="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -k 10 300 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?  # page in torch first
i=0
for P in "$P3" "$P1" "$P2"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmcta$i -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/pmcta$i.log 2>&1)
  rc=$?
  echo "pass $i exit $rc"; tail -2 gpurun_out/pmcta$i.log
  [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_summary.py gpurun_out/pmcta1 gpurun_out/pmcta2 gpurun_out/pmcta3 > gpurun_out/pmcta_summary.txt 2>&1
head -70 gpurun_out/pmcta_summary.txt
