# graph mode cost at N=1: one full-step graph vs per-bucket segment graphs (the N>1 mode) vs eager
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CS744_TUNE_CACHE=gpurun_out/tune_graphmode.json
for g in full segments none; do
  timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 --graph $g > gpurun_out/bench_graph_$g.log 2>&1 || exit $?
  echo "graph=$g $(tail -1 gpurun_out/bench_graph_$g.log | cut -c1-130)"
done
