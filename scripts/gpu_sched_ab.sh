set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for S in 0 1 2; do
  CS_CONV_SCHED=$S MICRO_SHAPES=0,1,2 timeout -k 10 300 python scripts/conv_microbench.py > gpurun_out/sched_$S.log 2>&1 || exit $?
done
grep -h tflops gpurun_out/sched_*.log | python -c "
import sys, json
rows=[json.loads(l) for l in sys.stdin]
for r in sorted(rows, key=lambda r:(r['B'],r['H'],r['mode'],r['sched'])): print(r['sched'], r['B'], r['H'], r['mode'], r['tflops'], r['us'], r['bm'], r['bn'], r['bk'], r['splits'])"
