"""Split the L0 JoinTable gradient into its NIN and BN contributions (GPU vs oracle)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g; g.add_path()
import numpy as np, torch
import sparseconvnet as scn
from oracle.encoders import OracleEncoder
from wsss3d import EasyDict, MODEL_REGISTRY
from wsss3d.synthetic import make_batch
torch.manual_seed(7)
b = make_batch(1, 10, seed=11, spacing=0.05)
cfg = dict(m=32, dimension=3, full_scale=4096, block_reps=2, residual_blocks=True)
model = MODEL_REGISTRY.get('SparseConvUNet')[0]('SparseConvUNet', **cfg).cuda()
ref = OracleEncoder('SparseConvUNet', **cfg).double(); ref.load_state_dict({k: v.double().cpu() for k, v in model.state_dict().items()})
cap = {'g': {}, 'o': {}}
names = ['encoder.2.5', 'encoder.2.6.0', 'encoder.2.6.1.0', 'encoder.2.3', 'encoder.2.4.1.0', 'encoder.2.4.1.4']
def hook(tag, mname):
    def f(mod, inp, out):
        cap[tag][mname] = out.features
        out.features.retain_grad()
    return f
for n1 in names:
    model.get_submodule(n1).register_forward_hook(hook('g', n1)); ref.get_submodule(n1).register_forward_hook(hook('o', n1))
c = torch.from_numpy(b['coords']); f = torch.from_numpy(b['feats'])
og = model(EasyDict(coords=c.cuda(), feature=f.cuda(), batch_offsets=b['batch_offsets']), istrain=True)
oo = ref(dict(coords=c, feature=f.double(), batch_offsets=b['batch_offsets']), istrain=True)
w = torch.linspace(-1, 1, og.shape[1])
(og * w.cuda()).sum().backward(retain_graph=True); (oo * w.double()).sum().backward(retain_graph=True)
loc = model.encoder[0]([c.cuda(), f.cuda()]).metadata  # fresh metadata only for locations of L0
tg = cap['g']['encoder.2.5']
# rebuild perm from an independent InputLayer on same coords (same Morton order)
lvl_loc = loc.locations(4096).cpu().numpy()
from oracle import scn_oracle as O
oi = O.InputLayer(3, 4096, mode=4)([c, f.double()])
idx = oi.metadata.levels[4096].lookup(lvl_loc); p = np.empty(len(idx), np.int64); p[idx] = np.arange(len(idx)); p = torch.from_numpy(p)
def cmp(name, a, bb):
    a = a.detach().double().cpu()[p]; bb = bb.detach()
    col = (a - bb).abs().max(0).values / (bb.abs().max() + 1e-30)
    print("%-32s max rel %.2e  cols0-31 %.2e cols32+ %.2e  |ref| %.3e" % (name, col.max().item(), col[:32].max().item(), col[32:].max().item() if col.numel() > 32 else -1, bb.abs().max().item()))
for n1 in names:
    cmp(n1 + ' out', cap['g'][n1], cap['o'][n1])
    cmp(n1 + ' grad', cap['g'][n1].grad, cap['o'][n1].grad)
J = 'encoder.2.5'
for br in ['encoder.2.6.0', 'encoder.2.6.1.0']:
    gg = torch.autograd.grad(cap['g'][br], cap['g'][J], grad_outputs=cap['g'][br].grad, retain_graph=True)[0]
    go = torch.autograd.grad(cap['o'][br], cap['o'][J], grad_outputs=cap['o'][br].grad, retain_graph=True)[0]
    cmp('dJoin via ' + br, gg, go)
