# round-2: channels-last ResNet path after the apply/finalize rewrite, split weight-gradient GEMM and
# 4-channel stem: GPU tests, ResNet-50 B=128 bench (bf16, fp32), kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cnn_nhwc_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_nhwc.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -15 gpurun_out/pytest_nhwc.log
[ $rc -eq 0 ] || exit $rc
for dt in bf16 fp32; do
  timeout -k 10 300 python bench.py --model resnet50 --dtype $dt --steps 10 --warmup 3 > gpurun_out/bench_rn50_nhwc_${dt}.log 2>&1 || exit $?
  echo "nhwc $dt: $(tail -1 gpurun_out/bench_rn50_nhwc_${dt}.log | cut -c1-200)"
done
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn50_nhwc -o run -- python3 $R/bench.py --model resnet50 --dtype bf16 --steps 5 --warmup 2 > $R/gpurun_out/prof_rn50_nhwc.log 2>&1) || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_rn50_nhwc --steps 7 > gpurun_out/prof_rn50_nhwc_summary.txt 2>&1
head -45 gpurun_out/prof_rn50_nhwc_summary.txt | cut -c1-180
