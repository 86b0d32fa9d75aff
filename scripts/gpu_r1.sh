set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/r1_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --engine torch --steps 30 --warmup 10 > gpurun_out/r1_bench_torch.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r1_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --engine torch --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r1_prof.log 2>&1
echo EXIT $?
