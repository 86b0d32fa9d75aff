# round-2: ResNet-50 (channels-last native path, bf16) per-GPU batch sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 128 256; do
  timeout -k 10 300 python bench.py --model resnet50 --dtype bf16 --batch-size $b --steps 10 --warmup 3 > gpurun_out/bench_rn50_b$b.log 2>&1 || exit $?
  echo "B=$b: $(tail -1 gpurun_out/bench_rn50_b$b.log | cut -c1-200)"
done
