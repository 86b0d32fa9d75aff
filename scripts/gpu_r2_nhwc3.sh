# round-2: NHWC gathers with 32-bit index math — channels-last tests, ResNet-50 bench (default B=256) and profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_cnn_nhwc_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_nhwc3.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/pytest_nhwc3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model resnet50 --dtype bf16 --steps 10 --warmup 3 > gpurun_out/bench_rn50_b256_idx32.log 2>&1 || exit $?
echo "B=256: $(tail -1 gpurun_out/bench_rn50_b256_idx32.log | cut -c1-200)"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn50_b256 -o run -- python3 $R/bench.py --model resnet50 --dtype bf16 --steps 4 --warmup 2 > $R/gpurun_out/prof_rn50_b256.log 2>&1) || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_rn50_b256 --steps 6 > gpurun_out/prof_rn50_b256_summary.txt 2>&1
grep -E "im2col|col2im|maxpool" gpurun_out/prof_rn50_b256_summary.txt | head -6 | cut -c1-160
