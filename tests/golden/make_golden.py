"""Generate the committed golden fixtures (run in the build container, where
/root/reference exists; the GPU box only reads the outputs).

topology.json
    For every encoder the reference registers and can construct, the
    state_dict (key, shape) list and parameter count produced by the
    REFERENCE'S OWN `models/SparseConvNet.py` (loaded unmodified by path) on
    top of the CPU oracle namespace injected as `sparseconvnet`, plus the
    reference registry's `embed_length(m)`.  This pins the module tree the
    product must reproduce (state_dict compatibility) and the oracle's
    builders.
oracle_<case>.npz
    Inputs (coords, feats), the seeded-init parameter checksum and fp64
    oracle outputs for small C1/C2/C3-shaped cases: sampled per-point
    features, scene features, and the gradient of a fixed scalar loss w.r.t.
    the first SubmanifoldConvolution weight plus per-parameter gradient sums.

Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(ROOT, "3d-weakly-supervised-semantic-segmentation_amd")
REF = "/root/reference"
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

from oracle import scn_oracle  # noqa: E402
from oracle.encoders import OracleEncoder  # noqa: E402
from wsss3d.edict import EasyDict  # noqa: E402
from wsss3d.synthetic import make_batch  # noqa: E402

TOPOLOGY_CASES = [
    ("SparseConvUNet", 16, 1, False), ("SparseConvUNet", 32, 2, True), ("SparseConvFCNet", 16, 1, False),
    ("SparseConvFCNet", 32, 1, False), ("SparseConvFCNetNarrow", 16, 1, False),
    ("SparseConvFCNetDirectUpPool", 32, 1, False), ("SparseConvFCNetDirectUpPoolLight", 32, 1, True),
]

# name, encoder, m, reps, residual, scenes, scale, spacing, seed
ORACLE_CASES = [
    ("c1_fcnencoder", "SparseConvFCNetEncoder", 16, 1, False, 1, 20, 0.1, 5),
    ("c2_unet_m16", "SparseConvUNet", 16, 1, False, 2, 20, 0.12, 6),
    ("c3_unet_m32_res", "SparseConvUNet", 32, 2, True, 1, 20, 0.12, 7),
]


def load_reference_models():
    """models/SparseConvNet.py from the reference, with the oracle as scn."""
    sys.modules["sparseconvnet"] = scn_oracle
    sys.modules["easydict"] = types.SimpleNamespace(EasyDict=EasyDict)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    spec = importlib.util.spec_from_file_location("reference_sparseconvnet_models",
                                                  os.path.join(REF, "models", "SparseConvNet.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    reg = importlib.import_module("utils.registry").MODEL_REGISTRY
    return mod, reg


def make_topology():
    mod, reg = load_reference_models()
    out = {}
    for name, m, reps, res in TOPOLOGY_CASES:
        cls, meta = reg.get(name)
        torch.manual_seed(0)
        enc = cls(name, m=m, dimension=3, full_scale=4096, block_reps=reps, residual_blocks=res)
        sd = enc.state_dict()
        out[f"{name}-m{m}-r{reps}-{int(res)}"] = {
            "embed_length": meta["embed_length"](m),
            "n_params": sum(p.numel() for p in enc.parameters()),
            "state_dict": [[k, list(v.shape)] for k, v in sd.items()],
        }
    with open(os.path.join(HERE, "topology.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("topology.json:", len(out), "encoders")


def oracle_case(tag, name, m, reps, res, scenes, scale, spacing, seed):
    b = make_batch(scenes, scale, seed=seed, spacing=spacing)
    torch.manual_seed(seed)
    ref = OracleEncoder(name, m=m, block_reps=reps, residual_blocks=res)
    checksum = float(sum(p.detach().double().sum() for p in ref.parameters()))
    ref = ref.double()
    coords = torch.from_numpy(b["coords"])
    feats = torch.from_numpy(b["feats"]).double()
    x = dict(coords=coords, feature=feats, batch_offsets=b["batch_offsets"])
    pp = ref(x)
    glob = ref(x, istrain=True)
    w = torch.linspace(-1, 1, glob.shape[1], dtype=torch.float64)
    (glob * w).sum().backward()
    rng = np.random.default_rng(seed)
    rows = np.sort(rng.choice(len(coords), size=min(256, len(coords)), replace=False))
    np.savez_compressed(
        os.path.join(HERE, f"oracle_{tag}.npz"),
        coords=b["coords"].astype(np.int16), feats=b["feats"], batch_offsets=np.array(b["batch_offsets"]),
        meta=np.array([name, str(m), str(reps), str(int(res)), str(seed)]),
        param_checksum=np.array(checksum), rows=rows, per_point=pp.detach().numpy()[rows],
        scene=glob.detach().numpy(), grad_first=ref.encoder[1].weight.grad.numpy(),
        grad_sums=np.array([p.grad.sum().item() for p in ref.parameters()]),
        grad_names=np.array([k for k, _ in ref.named_parameters()]),
        n_voxels=np.array(ref.encoder[0].forward([coords, feats]).features.shape[0]))
    print(f"oracle_{tag}.npz: {len(coords)} points")


if __name__ == "__main__":
    if os.path.isdir(REF):
        make_topology()
    else:
        print("reference not present: topology.json left as committed")
    for case in ORACLE_CASES:
        oracle_case(*case)
