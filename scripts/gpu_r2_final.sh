# round-2 final: attention vs SDPA table, full GPU suite, smoke, default bench (the driver's round-end steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -m cs744_pytorch_distributed_tutorial_amd.bench.attention --seq 2048 4096 8192 > gpurun_out/attn_vs_sdpa.log 2>&1 || exit $?
tail -8 gpurun_out/attn_vs_sdpa.log | cut -c1-250
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_shape.log 2>&1 || exit $?
tail -1 gpurun_out/bench_driver_shape.log | cut -c1-300
timeout -k 10 300 python bench.py --model llama3-8b --steps 4 --warmup 2 > gpurun_out/bench_llama_final.log 2>&1 || exit $?
tail -1 gpurun_out/bench_llama_final.log | cut -c1-200
timeout -k 10 300 python bench.py --model resnet50 --dtype bf16 --steps 10 --warmup 3 > gpurun_out/bench_rn50_final.log 2>&1 || exit $?
tail -1 gpurun_out/bench_rn50_final.log | cut -c1-200
