"""MultiLabelContrastive end to end on the device (BASELINE config 5 shape,
reduced): point branch through the fused tail, text branch, both losses."""
import pytest
import torch

from wsss3d import EasyDict, LOSS_REGISTRY, MODEL_REGISTRY
from wsss3d.encoders import segment_mean
from wsss3d.synthetic import make_batch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_multilabel_contrastive_step():
    torch.manual_seed(0)
    b = make_batch(3, 10, seed=2, spacing=0.05)
    pc = EasyDict(name="SparseConvFCNet", m=8, dimension=3, full_scale=4096, block_reps=1, residual_blocks=False)
    tc = EasyDict(name="TextTransformer", context_length=16, width=128, layers=1, vocab_size=64)
    cls, _ = MODEL_REGISTRY.get("MultiLabelContrastive")
    model = cls(pc, tc).to(DEV)
    x = EasyDict(coords=torch.from_numpy(b["coords"]).to(DEV), feature=torch.from_numpy(b["feats"]).to(DEV),
                 batch_offsets=b["batch_offsets"])
    text = torch.randint(1, 60, (2, 4, 16), device=DEV)
    text[..., -1] = 63
    has_text = torch.tensor([0, 2], device=DEV)
    logits, (gf, tf, ht) = model((x, (text, has_text)), istrain=True)
    assert logits.shape == (3, 20) and gf.shape == (3, 8 * 28) and tf.shape == (2, 4, 8 * 28)
    # scene features = the reference's per-scene mean of the per-point features
    with torch.no_grad():
        ref = segment_mean(model.pc_encoder(x), x.batch_offsets)
    assert (gf.detach() - ref).abs().max().item() <= 1e-5 * max(1.0, ref.abs().max().item())
    y = torch.from_numpy(b["scene_labels"]).to(DEV)
    loss = LOSS_REGISTRY.get("Classification")[0](logits, y) + LOSS_REGISTRY.get("TextContrastive")[0](gf, tf, ht)
    loss.backward()
    assert torch.isfinite(loss)
    assert model.text_encoder.token_embedding.weight.grad is not None
    assert model.pc_encoder.encoder[1].weight.grad.abs().sum() > 0


CAPTIONS = [
    "a brown wooden chair next to the table.", "a white door on the left wall.", "two monitors on the desk",
    "a bookshelf full of books", "the sofa is in front of the television", "a grey office chair",
    "kitchen cabinets above the counter", "a refrigerator to the right of the stove", "a toilet near the sink",
    "a bed with white pillows", "a shower curtain next to the bathtub", "a picture above the desk",
]


@pytest.mark.timeout(600)
def test_c5_shape_contrastive_parity():
    """BASELINE configs[4] per-GPU shape: MultiLabelContrastive = SparseConvFCNet m=32 r=1 at scale 20 +
    TextTransformer 512 wide, 12 layers, context 120, vocab 49408, captions through the fixed-shape
    tokenizer text_transform(120, 10), on four whole default-spacing scenes (the per-GPU workload of the
    8-GPU config is 8 such scenes; 4 keep the fp64 oracle's time bounded).  Scene features against the fp64
    oracle encoder and caption features against an fp64 copy of the text model, both at the 1e-4 bar; then the
    joint loss (Classification + TextContrastive, utils/loss.py:5-33) is back-propagated and every parameter
    gradient of the point branch is compared with the oracle's gradient for the same upstream gradient of the
    scene features, under the device run's ReLU decisions (oracle/parity.py), at 1e-3 of the tensor's max
    (models/MultiLabelContrastive.py:21-42)."""
    import copy
    from oracle.encoders import OracleEncoder
    from oracle.parity import run_shared_masks
    from wsss3d.tokenizer import text_transform
    torch.manual_seed(0)
    B = 4
    b = make_batch(B, 20, seed=4)
    pc = EasyDict(name="SparseConvFCNet", m=32, dimension=3, full_scale=4096, block_reps=1, residual_blocks=False)
    tc = EasyDict(name="TextTransformer", context_length=120, width=512, layers=12, vocab_size=49408)
    cls, _ = MODEL_REGISTRY.get("MultiLabelContrastive")
    model = cls(pc, tc).to(DEV)
    tt = text_transform(120, 10)
    text = torch.stack([tt(CAPTIONS[k:] + CAPTIONS[:k]) for k in (0, 3, 5, 8)]).to(DEV)
    assert text.shape == (B, 10, 120)
    has_text = torch.arange(B, device=DEV)
    x = EasyDict(coords=torch.from_numpy(b["coords"]).to(DEV), feature=torch.from_numpy(b["feats"]).to(DEV),
                 batch_offsets=b["batch_offsets"])
    logits, (gf, tf, ht) = model((x, (text, has_text)), istrain=True)
    assert logits.shape == (B, 20) and gf.shape == (B, 896) and tf.shape == (B, 10, 896)
    gf.retain_grad()

    ref = OracleEncoder("SparseConvFCNet", m=32, block_reps=1, residual_blocks=False).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in model.pc_encoder.state_dict().items()})
    xo = dict(coords=torch.from_numpy(b["coords"]), feature=torch.from_numpy(b["feats"]).double(),
              batch_offsets=b["batch_offsets"])

    tref = copy.deepcopy(model.text_encoder).double().cpu()
    lin = copy.deepcopy(model.text_linear).double().cpu()
    with torch.no_grad():
        tfr = lin(tref(text.view(-1, 120).cpu(), as_dict=True)["x"]).view(B, 10, -1)
    err = (tf.detach().double().cpu() - tfr).abs().max().item()
    assert err <= 1e-4 * max(1.0, tfr.abs().max().item()), err
    del tref, tfr

    y = torch.from_numpy(b["scene_labels"]).to(DEV)
    loss = LOSS_REGISTRY.get("Classification")[0](logits, y) + LOSS_REGISTRY.get("TextContrastive")[0](gf, tf, ht)
    loss.backward()
    assert torch.isfinite(loss)
    assert model.text_encoder.transformer.resblocks[11].mlp.c_proj.weight.grad.abs().sum() > 0
    upstream = gf.grad.detach().double().cpu()
    assert upstream.abs().max() > 0

    # the oracle forward with the device's ReLU decisions: a second device forward of the point branch (same
    # inputs, deterministic kernels: the same values and decisions as the training forward above)
    glob_g, gref, st = run_shared_masks(model.pc_encoder, ref, x, xo, istrain=True)
    assert torch.equal(glob_g.detach(), gf.detach()), "device encoder forward is not reproducible"
    assert st["max_flip_margin"] < 1e-4, st
    err = (gf.detach().double().cpu() - gref.detach()).abs().max().item()
    assert err <= 1e-4 * max(1.0, gref.abs().max().item()), err
    (gref * upstream).sum().backward()
    gg = dict(model.pc_encoder.named_parameters())
    n_cmp = 0
    for k, p in ref.named_parameters():
        g_dev = gg[k].grad
        assert g_dev is not None, k
        scale = max(p.grad.abs().max().item(), 1e-12)
        e = (g_dev.double().cpu() - p.grad).abs().max().item()
        assert e <= 1e-3 * scale + 1e-9, f"grad {k}: {e:.3e} vs scale {scale:.3e} ({st})"
        n_cmp += 1
    assert n_cmp == len(gg)


def test_text_block_fixture_on_device():
    """The reference ResidualAttentionBlock fixture (tests/golden/text_block.npz, fp64) reproduced by the
    text block on the device."""
    import json
    import os
    import numpy as np
    from wsss3d.text import ResidualAttentionBlock
    gold = os.path.join(os.path.dirname(__file__), "golden")
    g = np.load(os.path.join(gold, "text_block.npz"))
    meta = json.load(open(os.path.join(gold, "text_block_keys.json")))
    blk = ResidualAttentionBlock(meta["width"], meta["heads"]).double().to(DEV)
    blk.load_state_dict({k: torch.from_numpy(g["param/" + k]).double() for k in meta["keys"]})
    x = torch.from_numpy(g["x"]).double().transpose(0, 1).to(DEV)
    with torch.no_grad():
        y = blk(x).transpose(0, 1).cpu()
    assert (y - torch.from_numpy(g["y"])).abs().max().item() < 1e-10


@pytest.mark.parametrize("head", ["MultiLabel", "FullySupervised"])
def test_fused_eval_logits_match_per_point_head(head):
    """The fused eval head (heads.point_logits: Linear on the voxel rows, msp_point_rows_bias gather) against the
    reference's composition linear(pc_encoder(x)) on the same device model (train.py:106,
    models/MultiLabelContrastive.py:64-70, 96-99); FullySupervised's training outputs (scene-mean logits and
    per-point logits, :84-94) and every parameter gradient through the fused head's backward against the same
    composition.  Eval-mode BatchNorm (running statistics) for the eval call."""
    torch.manual_seed(1)
    b = make_batch(2, 20, seed=6, spacing=0.04)
    pc = EasyDict(name="SparseConvUNet", m=16, dimension=3, full_scale=4096, block_reps=1, residual_blocks=True)
    model = MODEL_REGISTRY.get(head)[0](pc).to(DEV)
    with torch.no_grad():
        model.linear.bias.uniform_(-0.5, 0.5)
    x = EasyDict(coords=torch.from_numpy(b["coords"]).to(DEV), feature=torch.from_numpy(b["feats"]).to(DEV),
                 batch_offsets=b["batch_offsets"])
    model.eval()
    with torch.no_grad():
        fused = model(x)
        ref = model.linear(model.pc_encoder(x))
    assert fused.shape == ref.shape == (len(b["coords"]), 20)
    err = (fused - ref).abs().max().item()
    assert err <= 1e-5 * max(1.0, ref.abs().max().item()), err
    if head != "FullySupervised":
        return
    model.train()
    y = torch.from_numpy(b["labels"]).to(DEV)
    y[::7] = -100
    up = torch.randn(2, 20, device=DEV)
    grads = []
    for fused_path in (True, False):
        model.zero_grad(set_to_none=True)
        if fused_path:
            glob, logits = model((x, None), istrain=True)
        else:
            logits = model.linear(model.pc_encoder(x))
            glob = segment_mean(logits, x.batch_offsets)
        loss = LOSS_REGISTRY.get("Classification")[0](logits, y) + (glob * up).sum()
        loss.backward()
        grads.append(({k: p.grad.detach().clone() for k, p in model.named_parameters()}, glob.detach(),
                      logits.detach()))
    (gf, globf, lf), (gr, globr, lr) = grads
    assert (globf - globr).abs().max().item() <= 1e-5 * max(1.0, globr.abs().max().item())
    assert (lf - lr).abs().max().item() <= 1e-5 * max(1.0, lr.abs().max().item())
    for k in gr:
        scale = max(gr[k].abs().max().item(), 1e-12)
        assert (gf[k] - gr[k]).abs().max().item() <= 1e-4 * scale + 1e-9, k


def test_device_logit_store_matches_cpu_index_add():
    """wsss3d.evaluate.PointLogitStore.add = train.py:107's `store.index_add_(0, point_ids, predictions.cpu())`
    bit for bit, over two validation reps (every id once per rep, shuffled, as valMerge's point_ids) and over
    a batch with repeated ids (the serial loop's order decides the rounding; the device sorts stably)."""
    from wsss3d.evaluate import PointLogitStore
    g = torch.Generator().manual_seed(3)
    n = 50000
    store_cpu = torch.zeros(n, 20)
    dev = PointLogitStore(n, DEV)
    for rep in range(2):
        for part in torch.randperm(n, generator=g).chunk(3):
            pred = torch.randn(len(part), 20, generator=g) * 10
            store_cpu.index_add_(0, part, pred)
            dev.add(part.to(DEV), pred.to(DEV))
    assert torch.equal(dev.cpu(), store_cpu)
    assert torch.equal(dev.argmax().cpu(), store_cpu.max(1)[1])
    ids = torch.randint(0, 300, (40000,), generator=g)
    src = torch.randn(40000, 20, generator=g) * torch.logspace(-3, 3, 40000)[:, None]
    base = torch.randn(300, 20, generator=g)
    want = base.clone().index_add_(0, ids, src)
    got = base.to(DEV)
    from sparseconvnet.ops import index_add_rows
    index_add_rows(got, ids.to(DEV), src.to(DEV))
    assert torch.equal(got.cpu(), want)
    with pytest.raises(IndexError):
        index_add_rows(got, torch.tensor([0, 300], device=DEV), src[:2].to(DEV))
