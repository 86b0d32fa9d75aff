"""Debug: compare native-engine activations / grads per block with an fp64 torch reference."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from cs744_pytorch_distributed_tutorial_amd.models import VGG11
from cs744_pytorch_distributed_tutorial_amd.utils import data as dm
from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
tr = NativeTrainer(batch_size=B, device=dev, train_size=256, test_size=40, autotune=False, graph="none")
ref = VGG11().double()
ref.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in tr.state_dict().items()})
idx = torch.tensor(tr.sampler.indices()[:B])
x = dm.augment_reference(tr.train_set.data, idx, tr.aug_train.cpu()).double()
y = tr.train_set.targets[idx]
acts = {}
h = x
for i, m in enumerate(ref.layers):
    h = m(h)
    if isinstance(m, torch.nn.Conv2d):
        h.retain_grad()
        acts[i] = h
h.retain_grad()
feat = h
out = ref.fc1(h.view(B, -1))
loss = F.cross_entropy(out, y)
loss.backward()
tr.step()
torch.cuda.synchronize()
print("loss", tr.last_loss(), loss.item())
def rel(a, b):
    a = a.double().cpu(); b = b.double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()
specs = tr.layout.specs
for l, s in enumerate(specs):
    yv = tr.engine.tensor(l, "y")[:B * s.hw * s.hw].view(B, s.hw, s.hw, s.cout).permute(0, 3, 1, 2)
    print(f"block {l} conv out rel err {rel(yv, acts[s.conv_idx]):.3e}")
g = tr.grads_state()
for n, p in ref.named_parameters():
    print(f"{n:20s} grad rel {rel(g[n], p.grad):.3e}")
