"""Layer-by-layer forward/backward error of the HIP encoder vs the fp64 oracle
(same module tree; rows mapped through the per-level site coordinates)."""
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
ref = OracleEncoder(name, **cfg).double(); ref.load_state_dict({k: v.double().cpu() for k, v in model.state_dict().items()})
ref32 = OracleEncoder(name, **cfg); ref32.load_state_dict({k: v.float().cpu() for k, v in model.state_dict().items()})
cap = {'g': {}, 'o': {}, 'f': {}}
order = []
def hook(tag, mname):
    def f(mod, inp, out):
        if isinstance(out, list) or not hasattr(out, 'features'): return
        if tag == 'g': order.append(mname)
        cap[tag][mname] = out
        if out.features.requires_grad:
            out.features.register_hook(lambda gr: cap[tag].__setitem__(mname + '#grad', gr))
    return f
for (n1, m1) in model.named_modules(): m1.register_forward_hook(hook('g', n1))
for (n1, m1) in ref.named_modules(): m1.register_forward_hook(hook('o', n1))
for (n1, m1) in ref32.named_modules(): m1.register_forward_hook(hook('f', n1))
c = torch.from_numpy(b['coords']); f = torch.from_numpy(b['feats'])
og = model(EasyDict(coords=c.cuda(), feature=f.cuda(), batch_offsets=b['batch_offsets']), istrain=True)
oo = ref(dict(coords=c, feature=f.double(), batch_offsets=b['batch_offsets']), istrain=True)
of = ref32(dict(coords=c, feature=f, batch_offsets=b['batch_offsets']), istrain=True)
w = torch.linspace(-1, 1, og.shape[1])
(og * w.cuda()).sum().backward(); (oo * w.double()).sum().backward(); (of * w).sum().backward()
perms = {}
def perm_for(tg, to):
    size = int(tg.spatial_size[0])
    if size not in perms:
        loc = tg.metadata.locations(size).cpu().numpy()
        idx = to.metadata.levels[size].lookup(loc)
        p = np.empty(len(idx), np.int64); p[idx] = np.arange(len(idx)); perms[size] = torch.from_numpy(p)
    return perms[size]
for mname in order:
    tg, to = cap['g'][mname], cap['o'].get(mname)
    if to is None: continue
    p = perm_for(tg, to)
    a = tg.features.detach().double().cpu()[p]; bb = to.features.detach()
    e = ((a - bb).abs().max() / (bb.abs().max() + 1e-30)).item()
    e32 = ((cap['f'][mname].features.detach().double() - bb).abs().max() / (bb.abs().max() + 1e-30)).item()
    ge = float('nan')
    if mname + '#grad' in cap['g'] and mname + '#grad' in cap['o']:
        ga = cap['g'][mname + '#grad'].double().cpu()[p]; gb = cap['o'][mname + '#grad']
        ge = ((ga - gb).abs().max() / (gb.abs().max() + 1e-30)).item()
    ge32 = float('nan')
    if mname + '#grad' in cap['f'] and mname + '#grad' in cap['o']:
        ge32 = ((cap['f'][mname + '#grad'].double() - cap['o'][mname + '#grad']).abs().max() / (cap['o'][mname + '#grad'].abs().max() + 1e-30)).item()
    print("%-44s %-24s size %5d V %7d  fwd %.2e (cpu32 %.2e)  grad %.2e (cpu32 %.2e)" % (mname[-44:], type(model.get_submodule(mname)).__name__, int(tg.spatial_size[0]), a.shape[0], e, e32, ge, ge32))
