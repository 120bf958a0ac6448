import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g; g.add_path()
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
from test_gpu_encoders import _models, CASES
from oracle.parity import run_shared_masks
case = [c for c in CASES if c[0] == sys.argv[1]][0]
model, ref, xg, xo = _models(*case)
for it, ist in enumerate([False, True, True, False]):
    og, oo, st = run_shared_masks(model, ref, xg, xo, istrain=ist)
    d = (og.detach().double().cpu() - oo.detach()).abs()
    print(it, ist, "err", d.max().item(), "max", oo.abs().max().item(), st, "worst col", d.max(0).values.argmax().item() if d.dim() == 2 else None)
with torch.no_grad():
    d = (model(xg, istrain=True).double().cpu() - ref(xo, istrain=True)).abs()
    print("free run glob", d.max().item())
