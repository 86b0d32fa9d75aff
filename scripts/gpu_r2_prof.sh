# round-2 kernel profile of the default bench config (shipped tiles, side-stream wgrad) and of
# the serial backward: rocprofv3 kernel trace -> per-kernel tables in gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for tag in ovl serial; do
  if [ $tag = serial ]; then export CS_OVERLAP_WGRAD=0; fi
  timeout -k 10 240 python3 bench.py --steps 200 --warmup 30 > gpurun_out/bench_r2p_$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_r2p_$tag.log
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r2_$tag -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof_r2_$tag.log 2>&1) || exit $?
  python3 scripts/prof_summary.py gpurun_out/prof_r2_$tag --steps 25 --timeline 90 > gpurun_out/prof_r2_${tag}_summary.txt 2>&1
  head -45 gpurun_out/prof_r2_${tag}_summary.txt
done
