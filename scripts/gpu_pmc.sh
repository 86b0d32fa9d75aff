# usage: bash scripts/gpu_pmc.sh  — PMC counter passes (one rocprofv3 run per pass) over a short tuned bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export CS744_TUNE_CACHE=$R/scripts/tune_vgg11_b64.json
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc$i -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/pmc$i.log 2>&1
  rc=$?
  cd $R
  echo "pass $i exit $rc"; tail -2 gpurun_out/pmc$i.log
  [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 > gpurun_out/pmc_summary.txt 2>&1
cat gpurun_out/pmc_summary.txt | head -60
