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
