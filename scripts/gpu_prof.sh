# usage: bash scripts/gpu_prof.sh TAG [bench args...]  — tunes once, then a rocprofv3 kernel trace of the tuned run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-native}
shift
export CS744_TUNE_CACHE=$R/gpurun_out/tune_$TAG.json
timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 "$@" > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$TAG.log
python3 -c "
import json;d=json.load(open('$CS744_TUNE_CACHE'));k=list(d)[0];print(k)
for t,u in zip(d[k]['tiles'],[x for x in d[k]['us'] if x>0]): print(t, round(u,2))" || true
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 20 --warmup 5 "$@" > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?
cd $R
echo "rocprof exit $rc"; tail -1 gpurun_out/prof_$TAG.log
python3 scripts/prof_summary.py gpurun_out/prof_$TAG --steps 25 --timeline 70 > gpurun_out/prof_${TAG}_summary.txt 2>&1; head -40 gpurun_out/prof_${TAG}_summary.txt
exit $rc
