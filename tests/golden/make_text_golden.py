"""Golden fixture for the text branch (run in the build container, where the
reference is readable; the fixture is committed, the reference is not read at
test time).  Loads the reference's own `models/utils.py` by path (it imports
only torch / collections), builds its ResidualAttentionBlock with the causal
additive mask of `models/Transformer.py:88-94`, and records the parameters,
an input and the block output, plus the block's state_dict key names.

    python tests/golden/make_text_golden.py [/root/reference]
"""
import importlib.util
import json
import os
import sys

import numpy as np
import torch

ref_root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
spec = importlib.util.spec_from_file_location("ref_models_utils", os.path.join(ref_root, "models", "utils.py"))
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)

torch.manual_seed(0)
L, B, D, H = 10, 2, 128, 2
mask = torch.empty(L, L).fill_(float("-inf")).triu_(1)
blk = mod.ResidualAttentionBlock(D, H, mask)
with torch.no_grad():
    for p in blk.parameters():
        p.normal_(0, 0.2)
x = torch.randn(L, B, D)  # the reference works on (L, B, D)
# stored in f32, evaluated in f64 on those exact values
out = {f"param/{k}": v.detach().numpy() for k, v in blk.state_dict().items()}
out["x"] = x.numpy()
blk = blk.double()
y = blk(x.double())
out["y"] = y.detach().numpy()
here = os.path.dirname(os.path.abspath(__file__))
np.savez_compressed(os.path.join(here, "text_block.npz"), **out)
with open(os.path.join(here, "text_block_keys.json"), "w") as f:
    json.dump({"heads": H, "width": D, "keys": list(blk.state_dict().keys())}, f, indent=1)
print("wrote text_block.npz", {k: v.shape for k, v in out.items()})
