"""HIP path against the committed fp64 oracle fixtures (tests/golden/).

The product model is built with the fixture's seed: its construction order
matches the oracle's (tests/test_host.py::test_seeded_init_equals_oracle), so
the parameter checksum must equal the fixture's before anything is compared.
Per-point features (sampled rows) and scene features within 1e-4 of the
fixture (relative to max(1, |value|)).  The first-layer weight gradient is a
free-running comparison (the fixture fixes the fp64 ReLU decisions, the
device takes its own fp32 ones; see tests/test_gpu_encoders.py for the
shared-decision check at 1e-3 per element): its relative Frobenius error
must stay below 1e-2."""
import os

import numpy as np
import pytest
import torch

import sparseconvnet as scn  # noqa: F401
from wsss3d import EasyDict, MODEL_REGISTRY

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("tag", ["c1_fcnencoder", "c2_unet_m16", "c3_unet_m32_res"])
def test_hip_matches_golden(tag):
    z = np.load(os.path.join(GOLD, f"oracle_{tag}.npz"))
    name, m, reps, res, seed = z["meta"].tolist()
    torch.manual_seed(int(seed))
    model = MODEL_REGISTRY.get(name)[0](name, m=int(m), dimension=3, full_scale=4096, block_reps=int(reps),
                                        residual_blocks=bool(int(res)))
    chk = float(sum(p.detach().double().sum() for p in model.parameters()))
    assert abs(chk - float(z["param_checksum"])) < 1e-9 * max(1.0, abs(chk))
    model = model.cuda()
    x = EasyDict(coords=torch.from_numpy(z["coords"].astype(np.int64)).cuda(),
                 feature=torch.from_numpy(z["feats"]).cuda(), batch_offsets=z["batch_offsets"].tolist())
    pp = model(x)
    t = model.encoder[0]([x.coords, x.feature])
    assert t.features.shape[0] == int(z["n_voxels"])
    glob = model(x, istrain=True)
    (glob * torch.linspace(-1, 1, glob.shape[1]).cuda()).sum().backward()
    got = pp.detach().double().cpu().numpy()[z["rows"]]
    assert np.abs(got - z["per_point"]).max() <= 1e-4 * max(1.0, np.abs(z["per_point"]).max())
    assert np.abs(glob.detach().double().cpu().numpy() - z["scene"]).max() <= 1e-4
    g = model.encoder[1].weight.grad.double().cpu().numpy()
    assert np.linalg.norm(g - z["grad_first"]) <= 1e-2 * np.linalg.norm(z["grad_first"])
