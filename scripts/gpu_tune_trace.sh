# kernel trace of a fresh autotune: GEMM-only time of every (tile, split, staging) candidate
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/tunetrace -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/tunetrace.log 2>&1
rc=$?; cd $R; echo "rocprof exit $rc"; tail -1 gpurun_out/tunetrace.log | cut -c1-150; exit $rc
