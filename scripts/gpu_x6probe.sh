# X6 split cost probe: x6-only autotune with the real split vs a split-free build (wrong numbers).
# Needs _probe_C.so in the repo root: the package linked with conv_gemm.hip built with -DCS_X6_PROBE=1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CS_CONV_MATH=1 CS744_TUNE_CACHE=gpurun_out/tune_x6only.json timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 > gpurun_out/bench_x6only.log 2>&1 || exit $?
tail -1 gpurun_out/bench_x6only.log | cut -c1-120
cp _probe_C.so cs744_pytorch_distributed_tutorial_amd/_C.so
CS_CONV_MATH=1 CS744_TUNE_CACHE=gpurun_out/tune_x6probe.json timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 > gpurun_out/bench_x6probe.log 2>&1 || exit $?
tail -1 gpurun_out/bench_x6probe.log | cut -c1-120
