"""Per-parameter gradient error of the HIP encoder vs the fp64 and fp32 oracles."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g; g.add_path()
import numpy as np, torch
import sparseconvnet as scn
from oracle.encoders import OracleEncoder
from wsss3d import EasyDict, MODEL_REGISTRY
from wsss3d.synthetic import make_batch
name, m, reps, res = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), bool(int(sys.argv[4]))
torch.manual_seed(7)
b = make_batch(1, 10, seed=11, spacing=0.05)
cfg = dict(m=m, dimension=3, full_scale=4096, block_reps=reps, residual_blocks=res)
model = MODEL_REGISTRY.get(name)[0](name, **cfg).cuda()
sd = model.state_dict()
c = torch.from_numpy(b['coords']); f = torch.from_numpy(b['feats'])
res_ = {}
for tag, dt in [('64', torch.float64), ('32', torch.float32)]:
    r = OracleEncoder(name, **cfg).to(dt); r.load_state_dict({k: v.to(dt).cpu() for k, v in sd.items()})
    x = dict(coords=c, feature=f.to(dt), batch_offsets=b['batch_offsets'])
    o = r(x, istrain=True); w = torch.linspace(-1, 1, o.shape[1], dtype=dt); (o * w).sum().backward()
    res_[tag] = (o.detach().double(), {k: p.grad.double() for k, p in r.named_parameters()})
x = EasyDict(coords=c.cuda(), feature=f.cuda(), batch_offsets=b['batch_offsets'])
o = model(x, istrain=True); w = torch.linspace(-1, 1, o.shape[1]).cuda(); (o * w).sum().backward()
og = o.detach().double().cpu()
print("glob err gpu", (og - res_['64'][0]).abs().max().item(), "cpu32", (res_['32'][0] - res_['64'][0]).abs().max().item())
rows = []
for k, p in model.named_parameters():
    a = res_['64'][1][k]; s = a.abs().max().item() + 1e-30
    rows.append((((p.grad.double().cpu() - a).abs().max().item()) / s, ((res_['32'][1][k] - a).abs().max().item()) / s, k, tuple(p.shape)))
rows.sort(reverse=True)
for r_ in rows[:25]: print("%.3e  cpu32 %.3e  %s %s" % r_)
print("median gpu", np.median([r_[0] for r_ in rows]), "median cpu32", np.median([r_[1] for r_ in rows]))
