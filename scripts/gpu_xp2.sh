#!/bin/bash
# XP conv GEMMs: graph-timed sweep vs the tuned kernels, then two counter passes on a few configs
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 500 python -u scripts/xp_bench.py 64 10 > gpurun_out/xp_bench2.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/xp_bench2.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/xppmc$i -o run -- python3 $R/scripts/xp_pmc.py > $R/gpurun_out/xppmc$i.log 2>&1)
  rc=$?; echo "pass $i exit $rc"; tail -2 gpurun_out/xppmc$i.log
  [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_summary.py gpurun_out/xppmc1 gpurun_out/xppmc2 > gpurun_out/xppmc_summary.txt 2>&1
cat gpurun_out/xppmc_summary.txt | head -40
