# round-2: finish the TunableOp GEMM table of the Llama-3-8B step (seeded with the 5 forward shapes
# tuned by the first run); the watchdog (< timeout) ends an overrun cleanly so the table is written
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cp scripts/seed/tunableop_llama3_8b0.csv gpurun_out/tunableop_llama3_8b0.csv
(while sleep 50; do echo "[tick] $(date +%T)"; done) &
TICK=$!
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$GRAFT_REPO_ROOT/gpurun_out/tunableop_llama3_8b.csv \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=15 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=8 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=3 \
  timeout -k 10 1080 python bench.py --model llama3-8b --steps 1 --warmup 1 --watchdog-s 1000 > gpurun_out/tune2_llama.log 2>&1
rc=$?; kill $TICK; echo "tune exit $rc"; tail -2 gpurun_out/tune2_llama.log | cut -c1-250
wc -l gpurun_out/tunableop_llama3_8b0.csv
