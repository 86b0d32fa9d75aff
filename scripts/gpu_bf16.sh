# bf16 conv operands: numerics (conv + engine), then bench fp32 vs --dtype bf16
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_native_engine_gpu.py -k bf16 -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_bf16.log; [ $rc -eq 0 ] || exit $rc
export CS744_TUNE_CACHE=gpurun_out/tune_bf16.json
for d in bf16 fp32; do
  timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 --dtype $d > gpurun_out/bench_dtype_$d.log 2>&1 || exit $?
  echo "$d $(tail -1 gpurun_out/bench_dtype_$d.log | cut -c1-140)"
done
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --dtype bf16 --batch-size 256 > gpurun_out/bench_dtype_bf16_256.log 2>&1 || exit $?
echo "bf16 B=256 $(tail -1 gpurun_out/bench_dtype_bf16_256.log | cut -c1-140)"
