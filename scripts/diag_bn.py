"""Inspect one BatchNorm's backward inside the full UNet (GPU vs fp64 oracle)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g; g.add_path()
import numpy as np, torch
import sparseconvnet as scn
from oracle.encoders import OracleEncoder
from oracle import scn_oracle as O
from wsss3d import EasyDict, MODEL_REGISTRY
from wsss3d.synthetic import make_batch
BN = sys.argv[1] if len(sys.argv) > 1 else 'encoder.2.6.1.0'
torch.manual_seed(7)
b = make_batch(1, 10, seed=11, spacing=0.05)
cfg = dict(m=32, dimension=3, full_scale=4096, block_reps=2, residual_blocks=True)
model = MODEL_REGISTRY.get('SparseConvUNet')[0]('SparseConvUNet', **cfg).cuda()
ref = OracleEncoder('SparseConvUNet', **cfg).double(); ref.load_state_dict({k: v.double().cpu() for k, v in model.state_dict().items()})
cap = {}
def hook(tag):
    def f(mod, inp, out):
        x = inp[0].features; x.retain_grad(); out.features.retain_grad(); cap[tag] = (x, out.features)
    return f
model.get_submodule(BN).register_forward_hook(hook('g')); ref.get_submodule(BN).register_forward_hook(hook('o'))
c = torch.from_numpy(b['coords']); f = torch.from_numpy(b['feats'])
og = model(EasyDict(coords=c.cuda(), feature=f.cuda(), batch_offsets=b['batch_offsets']), istrain=True)
oo = ref(dict(coords=c, feature=f.double(), batch_offsets=b['batch_offsets']), istrain=True)
w = torch.linspace(-1, 1, og.shape[1])
(og * w.cuda()).sum().backward(retain_graph=True); (oo * w.double()).sum().backward(retain_graph=True)
meta = model.encoder[0]([c.cuda(), f.cuda()]).metadata
oi = O.InputLayer(3, 4096, mode=4)([c, f.double()])
idx = oi.metadata.levels[4096].lookup(meta.locations(4096).cpu().numpy()); p = np.empty(len(idx), np.int64); p[idx] = np.arange(len(idx)); p = torch.from_numpy(p)
xg, yg = cap['g']; xo, yo = cap['o']
print("x.grad is None?", xg.grad is None)
X = xg.detach().double().cpu()[p]; GY = yg.grad.double().cpu()[p]
DXg = torch.autograd.grad(yg, xg, grad_outputs=yg.grad, retain_graph=True)[0].double().cpu()[p]
Xo = xo.detach(); GYo = yo.grad
DXo = torch.autograd.grad(yo, xo, grad_outputs=yo.grad, retain_graph=True)[0]
print("BN-only dx: gpu vs oracle max err", (DXg - DXo).abs().max().item())
print("x err", (X - Xo).abs().max().item(), "gy err", (GY - GYo).abs().max().item(), "|gy|", GYo.abs().max().item())
# fp64 recompute of BN backward from the GPU's own x and gy
bnm = ref.get_submodule(BN)
wgt = bnm.weight.detach(); V = X.shape[0]
mu = X.mean(0); var = X.var(0, unbiased=False); inv = 1 / torch.sqrt(var + 1e-4)
xh = (X - mu) * inv; z = xh * wgt + bnm.bias.detach()
dz = torch.where(z > 0, GY, GY * bnm.leak)
dx = wgt * inv * (dz - dz.mean(0) - xh * (dz * xh).mean(0))
err_g = (DXg - dx).abs().max(0).values; err_o = (DXo - dx).abs().max(0).values
print("|dx| max", dx.abs().max().item())
for cc in torch.argsort(err_g, descending=True)[:6].tolist():
    zc = z[:, cc]
    print(f"ch {cc}: gpu err {err_g[cc]:.3e} oracle err {err_o[cc]:.3e} mean {mu[cc]:.4e} std {var[cc].sqrt():.4e} invstd {inv[cc]:.3e} "
          f"w {wgt[cc]:.3f} min|z| {zc.abs().min():.3e} frac z>0 {(zc>0).double().mean():.3f} |dx_c| {dx[:,cc].abs().max():.3e}")
    r = (DXg[:, cc] - dx[:, cc]).abs().argmax().item()
    print(f"   worst row {r}: x {X[r,cc]:.6e} z {z[r,cc]:.4e} gy {GY[r,cc]:.4e} dx_gpu {DXg[r,cc]:.6e} dx_ref {dx[r,cc]:.6e}")
