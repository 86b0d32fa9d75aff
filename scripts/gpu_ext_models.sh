# BASELINE.json extension configs on one MI355X: ResNet-50 ImageNet-shape, Llama-3 8B bf16, tiny LM
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MIOPEN_FIND_MODE=FAST
timeout -k 10 300 python bench.py --model resnet50 --dtype bf16 --steps 20 --warmup 5 > gpurun_out/bench_resnet50.log 2>&1 || exit $?
tail -1 gpurun_out/bench_resnet50.log | cut -c1-400
timeout -k 10 300 python bench.py --model llama-tiny --dtype bf16 --steps 20 --warmup 5 > gpurun_out/bench_llama_tiny.log 2>&1 || exit $?
tail -1 gpurun_out/bench_llama_tiny.log | cut -c1-400
timeout -k 10 400 python bench.py --model llama3-8b --dtype bf16 --batch-size 1 --seq-len 2048 --steps 5 --warmup 2 > gpurun_out/bench_llama8b.log 2>&1 || exit $?
tail -1 gpurun_out/bench_llama8b.log | cut -c1-400
