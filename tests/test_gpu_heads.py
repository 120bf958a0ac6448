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


def test_c5_shape_contrastive_parity():
    """BASELINE configs[4] per-GPU shape: MultiLabelContrastive = SparseConvFCNet m=32 r=1 at scale 20 +
    TextTransformer 512 wide, 12 layers, context 120, vocab 49408, captions through the fixed-shape
    tokenizer text_transform(120, 10).  Scene features against the fp64 oracle encoder and caption features
    against an fp64 copy of the text model, both at the 1e-4 bar; both losses back-propagate."""
    import copy
    from oracle.encoders import OracleEncoder
    from wsss3d.tokenizer import text_transform
    torch.manual_seed(0)
    b = make_batch(2, 20, seed=4, spacing=0.05)
    pc = EasyDict(name="SparseConvFCNet", m=32, dimension=3, full_scale=4096, block_reps=1, residual_blocks=False)
    tc = EasyDict(name="TextTransformer", context_length=120, width=512, layers=12, vocab_size=49408)
    cls, _ = MODEL_REGISTRY.get("MultiLabelContrastive")
    model = cls(pc, tc).to(DEV)
    tt = text_transform(120, 10)
    text = torch.stack([tt(CAPTIONS[k:] + CAPTIONS[:k]) for k in (0, 5)]).to(DEV)
    assert text.shape == (2, 10, 120)
    has_text = torch.arange(2, device=DEV)
    x = EasyDict(coords=torch.from_numpy(b["coords"]).to(DEV), feature=torch.from_numpy(b["feats"]).to(DEV),
                 batch_offsets=b["batch_offsets"])
    logits, (gf, tf, ht) = model((x, (text, has_text)), istrain=True)
    assert logits.shape == (2, 20) and gf.shape == (2, 896) and tf.shape == (2, 10, 896)

    ref = OracleEncoder("SparseConvFCNet", m=32, block_reps=1, residual_blocks=False).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in model.pc_encoder.state_dict().items()})
    with torch.no_grad():
        gref = ref(dict(coords=torch.from_numpy(b["coords"]), feature=torch.from_numpy(b["feats"]).double(),
                        batch_offsets=b["batch_offsets"]), istrain=True)
    err = (gf.detach().double().cpu() - gref).abs().max().item()
    assert err <= 1e-4 * max(1.0, gref.abs().max().item()), err

    tref = copy.deepcopy(model.text_encoder).double().cpu()
    lin = copy.deepcopy(model.text_linear).double().cpu()
    with torch.no_grad():
        tfr = lin(tref(text.view(-1, 120).cpu(), as_dict=True)["x"]).view(2, 10, -1)
    err = (tf.detach().double().cpu() - tfr).abs().max().item()
    assert err <= 1e-4 * max(1.0, tfr.abs().max().item()), err

    y = torch.from_numpy(b["scene_labels"]).to(DEV)
    loss = LOSS_REGISTRY.get("Classification")[0](logits, y) + LOSS_REGISTRY.get("TextContrastive")[0](gf, tf, ht)
    loss.backward()
    assert torch.isfinite(loss)
    assert model.text_encoder.transformer.resblocks[11].mlp.c_proj.weight.grad.abs().sum() > 0
    assert model.pc_encoder.encoder[1].weight.grad.abs().sum() > 0


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
