# round-2: PyTorch TunableOp (hipBLASLt + rocBLAS solution search per GEMM shape) for the Llama-3-8B step:
# tune once into a CSV, then time the step reading the table with tuning off
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
(while sleep 50; do echo "[tick] $(date +%T) $(wc -l < gpurun_out/tunableop_llama3_8b.csv 2>/dev/null)"; done) &
TICK=$!
export PYTORCH_TUNABLEOP_FILENAME=$GRAFT_REPO_ROOT/gpurun_out/tunableop_llama3_8b.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=50 \
  timeout -k 10 700 python bench.py --model llama3-8b --steps 1 --warmup 1 > gpurun_out/tune_llama.log 2>&1
rc=$?; kill $TICK; echo "tune exit $rc"; tail -2 gpurun_out/tune_llama.log | cut -c1-250
[ $rc -eq 0 ] || exit $rc
wc -l $PYTORCH_TUNABLEOP_FILENAME
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python bench.py --model llama3-8b --steps 4 --warmup 2 > gpurun_out/bench_llama_tuned.log 2>&1 || exit $?
echo "tuned: $(tail -1 gpurun_out/bench_llama_tuned.log | cut -c1-200)"
timeout -k 10 300 python bench.py --model llama3-8b --steps 4 --warmup 2 > gpurun_out/bench_llama_default.log 2>&1 || exit $?
echo "default: $(tail -1 gpurun_out/bench_llama_default.log | cut -c1-200)"
