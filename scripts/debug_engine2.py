"""Debug: partial backward (blocks 7..3) and inspect dz / gradient buffers vs fp64 autograd."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from cs744_pytorch_distributed_tutorial_amd.models import VGG11
from cs744_pytorch_distributed_tutorial_amd.utils import data as dm
from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn

dev = torch.device("cuda", 0)
B = 8
tr = NativeTrainer(batch_size=B, device=dev, train_size=256, test_size=40, autotune=False, graph="none")
ref = VGG11().double()
ref.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in tr.state_dict().items()})
idx = torch.tensor(tr.sampler.indices()[:B])
x = dm.augment_reference(tr.train_set.data, idx, tr.aug_train.cpu()).double()
y = tr.train_set.targets[idx]
acts, ins = {}, {}
h = x
for i, m in enumerate(ref.layers):
    if isinstance(m, torch.nn.Conv2d) and i > 0:
        h = h * 1.0
        h.retain_grad()
        ins[i] = h
    h = m(h)
    if isinstance(m, torch.nn.Conv2d):
        h.retain_grad(); acts[i] = h
loss = F.cross_entropy(ref.fc1(h.view(B, -1)), y)
# chain grads manually through detached block inputs
loss.backward()
for i in sorted(ins, reverse=True):
    pass
def rel(a, b):
    a = a.double().cpu(); b = b.double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()
tr._load_next_batch()
tr.engine.forward_train(B)
tr.engine.backward(7, 3, B)
torch.cuda.synchronize()
for l in range(4):
    print(l, [tr.engine.get_tile(l, m) for m in range(3)])
# block 3 = layers.11 conv (256->256 @8x8); its dz = grad wrt acts[11]
dz = tr.engine.tensor(0, "dz")[:B * 64 * 256].view(B, 8, 8, 256).permute(0, 3, 1, 2)
print("dz3 rel", rel(dz, acts[11].grad))
G2 = tr.engine.tensor(0, "g1")[:B * 64 * 256].view(B, 8, 8, 256).permute(0, 3, 1, 2)
print("G2 (grad of block-3 input) rel", rel(G2, ins[11].grad))
# recompute the dgrad standalone with several tiles
w3 = tr.layout.view(tr.params, "layers.11.weight").permute(0, 2, 3, 1).contiguous()
dzn = tr.engine.tensor(0, "dz")[:B * 64 * 256].view(-1, 256).clone()
for tile in [(64, 64, 1), (64, 64, 4), (64, 64, 16), (128, 128, 1), (64, 64, 8)]:
    dx = Fn.conv_dgrad(dzn, w3, B, 8, 8, bm=tile[0], bn=tile[1], splits=tile[2]).view(B, 8, 8, 256).permute(0, 3, 1, 2)
    print("standalone dgrad", tile, rel(dx, ins[11].grad))

# ---- isolate block 2's BN backward inside the engine
tr2 = NativeTrainer(batch_size=B, device=dev, train_size=256, test_size=40, autotune=False, graph="none")
tr2._load_next_batch()
tr2.engine.forward_train(B)
tr2.engine.backward(7, 2, B)
torch.cuda.synchronize()
C, H = 256, 8
M = B * H * H
y2 = tr2.engine.tensor(2, "y")[:M].double().cpu()
bn = tr2.engine.tensor(2, "bn").double().cpu()
G2 = tr2.engine.tensor(0, "g1")[:M * C].view(M, C).double().cpu()
sc, sh, mu, inv = bn[0], bn[1], bn[2], bn[3]
print("engine mean vs y2 mean", rel(mu, y2.mean(0)), "invstd", rel(inv, 1 / torch.sqrt(y2.var(0, unbiased=False) + 1e-5)))
z = torch.clamp(y2 * sc + sh, min=0)
g = torch.where(z > 0, G2, torch.zeros_like(G2))
xh = (y2 - mu) * inv
gd = tr2.grads_state()
print("dbeta rel", rel(gd["layers.9.bias"], g.sum(0)), "dgamma rel", rel(gd["layers.9.weight"], (g * xh).sum(0)))
print("sum|g|", g.abs().sum(0)[:4], "sum g", g.sum(0)[:4], "engine", gd["layers.9.bias"][:4])
n_zero = (y2 * sc + sh == 0).sum().item()
print("exact zeros in pre-relu", n_zero)
