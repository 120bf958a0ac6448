"""Full-size parity of the benchmarked networks (BASELINE.json configs[1] and configs[2] shapes at 2 cm,
whole synthetic scenes): the HIP path against the fp64 CPU oracle with shared ReLU decisions
(oracle/parity.py), at the sizes where the production kernel selections take over -- the dense row-group
convolution (msp_conv_nbr, >= 1e5 rows and c_out >= 64: level 0's 32 -> 64 backward-data), the tile-local
convolution (msp_conv_local, 64+ channels from 4096 rows: levels 1-4), the NetworkInNetwork kernel
(msp_nin_gemm), the per-wave split-bf16 tile at level 0 (conv_x6r) and the chunk-local weight gradient
(msp_conv_wgrad_chunk, c_out >= 64) beside the pair-list one.  The test records which forms ran
(through the same hook bench.py times them with) and requires each to have fired.

Bars (tests/test_gpu_encoders.py explains them): per-point and scene features within 1e-4 of
max(1, |oracle|); every parameter gradient within 1e-3 of its tensor's max; ReLU decisions the fp64
oracle would take differently only at rounding level (|z| < 1e-4).

The fp64 oracle of the headline network on two full scenes (~5e5 points) takes ~45 s and ~50 GB of host
memory on 16 threads (the GPU box allows ~270 GB).  # (models/SparseConvNet.py:57-71)
"""
import pytest
import torch

import sparseconvnet as scn  # noqa: F401
from sparseconvnet import _lib, ops
from oracle.encoders import OracleEncoder
from oracle.parity import run_shared_masks
from wsss3d import EasyDict, MODEL_REGISTRY
from wsss3d.synthetic import make_batch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class _Kinds:
    """Recorder that only notes which kernel forms ran (sparseconvnet/ops.py _record)."""

    def __init__(self):
        self.kinds = {}

    def run(self, kind, flops, fn, nbytes=0):
        kind = kind.split("[")[0]  # without the shape tag of MI3DSPARSE_KIND_SHAPES=1
        self.kinds[kind] = self.kinds.get(kind, 0) + 1
        return fn()


def _close(a, b, tol, what):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    err = (a - b).abs().max().item()
    lim = tol * max(1.0, b.abs().max().item())
    print(f"{what}: max err {err:.3e} (bar {lim:.3e})")
    assert err <= lim, f"{what}: {err:.3e} > {lim:.3e}"
    return err


def _run(name, m, reps, residual, scenes, need, seed=17):
    torch.manual_seed(5)
    batch = make_batch(scenes, 50, seed=seed)  # whole rooms at 2 cm spacing, scale 50
    cfg = dict(m=m, dimension=3, full_scale=4096, block_reps=reps, residual_blocks=residual)
    cls, _ = MODEL_REGISTRY.get(name)
    model = cls(name, **cfg).to(DEV)
    ref = OracleEncoder(name, **cfg).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in model.state_dict().items()})
    coords = torch.from_numpy(batch["coords"])
    feats = torch.from_numpy(batch["feats"])
    xg = EasyDict(coords=coords.to(DEV), feature=feats.to(DEV), batch_offsets=batch["batch_offsets"])
    xo = dict(coords=coords, feature=feats.double(), batch_offsets=batch["batch_offsets"])
    rec = _Kinds()
    _lib.set_recorder(rec)
    try:
        with torch.no_grad():
            out_g, out_o, st0 = run_shared_masks(model, ref, xg, xo, istrain=False)
        _close(out_g, out_o, 1e-4, "per-point features")
        assert st0["max_flip_margin"] < 1e-4, st0
        del out_g, out_o
        glob_g, glob_o, st = run_shared_masks(model, ref, xg, xo, istrain=True)
        _close(glob_g, glob_o, 1e-4, "scene features")
        assert st["max_flip_margin"] < 1e-4, st
        w = torch.linspace(-1, 1, glob_o.shape[1], dtype=torch.float64)
        (glob_g * w.float().to(DEV)).sum().backward()
        (glob_o * w).sum().backward()
    finally:
        _lib.set_recorder(None)
    gg = dict(model.named_parameters())
    worst = 0.0
    for k, p in ref.named_parameters():
        g_gpu = gg[k].grad
        assert g_gpu is not None, k
        scale = max(p.grad.abs().max().item(), 1e-12)
        err = (g_gpu.double().cpu() - p.grad).abs().max().item()
        worst = max(worst, err / scale)
        assert err <= 1e-3 * scale + 1e-9, f"grad {k}: {err:.3e} vs scale {scale:.3e} ({st})"
    print(f"parameter gradients: worst max err / tensor max {worst:.3e} (bar 1e-3)")
    missing = [k for k in need if k not in rec.kinds]
    assert not missing, f"production forms that did not run: {missing} (ran: {sorted(rec.kinds)})"
    return rec.kinds


def test_headline_unet_full_size_parity():
    """configs[2] network (SparseConvUNet m=32, block_reps=2, residual) on two whole scenes at 2 cm:
    level 0 >= 2^18 voxels (fp32 NIN form, split form below), level 1 >= 1e5 (dense row groups)."""
    kinds = _run("SparseConvUNet", 32, 2, True, 2,
                 need=["subm_fwd/x6r", "subm_fwd/x6s", "subm_bwd_data/x6s", "subm_fwd/x6d",
                       "nin_fwd/f32", "nin_bwd_data/f32", "nin_fwd/x6", "nin_bwd_data/x6", "wgrad_strided/x6", "wgrad_deconv/x6", "wgrad/x6c", "nin_wgrad/x6", "conv_fwd/x6d",
                       "deconv_fwd/" + ops.PAIRS_FORM, "subm_fwd/f32n", "wgrad/f32n"])
    assert kinds["subm_fwd/x6s"] >= 4


@pytest.mark.timeout(900)
def test_c2_unet_full_size_parity():
    """configs[1] exactly as `bench.py --preset c2` runs it (rank 0's first batch: make_batch(4, 50, seed=0), all
    four scenes): SparseConvUNet m=16, block_reps=1, VGG blocks, forward and every parameter gradient."""
    _run("SparseConvUNet", 16, 1, False, 4, need=["subm_fwd/x6r", "subm_bwd_data/x6r", "wgrad/x6", "subm_fwd/f32n",
                                                  "wgrad/f32n"], seed=0)
