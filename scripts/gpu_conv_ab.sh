# conv kernel numerics + schedule A/B microbench + tuned bench (one GPU call)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_bn_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || exit $rc
for S in 0 1; do
  CS_CONV_SCHED=$S MICRO_SHAPES=${MICRO:-0,2,4} timeout -k 10 300 python scripts/conv_microbench.py > gpurun_out/sched_$S.log 2>&1 || exit $?
done
grep -h tflops gpurun_out/sched_*.log | python -c "
import sys, json
rows=[json.loads(l) for l in sys.stdin]
for r in sorted(rows, key=lambda r:(r['B'],r['H'],r['mode'],r['sched'])): print(r['sched'], r['B'], r['H'], r['cin'], r['mode'], r['tflops'], r['us'], r['bm'], r['bn'], r['bk'], r['splits'])"
export CS744_TUNE_CACHE=$GRAFT_REPO_ROOT/gpurun_out/tune_ab.json
timeout -k 10 300 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_ab.log 2>&1 || exit $?
tail -1 gpurun_out/bench_ab.log
