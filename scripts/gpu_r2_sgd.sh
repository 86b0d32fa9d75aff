# SGD pass A/B: original loop (1) vs U float4 groups per thread (4, 8): kernel time + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for u in 1 4 8; do
CS_SGD_UNROLL=$u timeout -k 10 60 python -c "
import torch
from cs744_pytorch_distributed_tutorial_amd.ops import native
C = native.C()
n = 9231168
p, g, m = (torch.randn(n, device='cuda') for _ in range(3))
for _ in range(20): C.sgd_flat(p, g, m, 0.1, 0.9, 1e-4, 0.0, 1.0, False)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
# interleave a 128 MB sweep so the buffers are not all L2-hot (as in the step)
x = torch.empty(32 << 20, device='cuda')
tot = 0.0
for _ in range(50):
    x.add_(1.0)
    e0.record(); C.sgd_flat(p, g, m, 0.1, 0.9, 1e-4, 0.0, 1.0, False); e1.record(); torch.cuda.synchronize()
    tot += e0.elapsed_time(e1)
print('unroll $u: sgd_flat %.1f us' % (1000 * tot / 50))
" 2>&1 | grep unroll || exit 1
done
for u in 1 4 8 1 4; do
CS_SGD_UNROLL=$u timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/sgd_bench.log 2>&1 || exit 1
echo "unroll $u bench: $(tail -1 gpurun_out/sgd_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
