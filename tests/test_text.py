"""Text branch (wsss3d/text.py) against the reference's own attention block
(fixture from tests/golden/make_text_golden.py: models/utils.py's
ResidualAttentionBlock with the causal additive mask, evaluated in fp64) and
the TextTransformer / TextContrastive contract.  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from wsss3d import EasyDict, LOSS_REGISTRY, MODEL_REGISTRY
from wsss3d.text import ResidualAttentionBlock, TextTransformer

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_block_matches_reference_fixture():
    g = np.load(os.path.join(GOLD, "text_block.npz"))
    meta = json.load(open(os.path.join(GOLD, "text_block_keys.json")))
    blk = ResidualAttentionBlock(meta["width"], meta["heads"]).double()
    # same state_dict layout as the reference block (checkpoints interchange)
    assert list(blk.state_dict().keys()) == meta["keys"]
    blk.load_state_dict({k: torch.from_numpy(g["param/" + k]).double() for k in meta["keys"]})
    x = torch.from_numpy(g["x"]).double().transpose(0, 1)  # reference (L, B, D) -> (B, L, D)
    y = blk(x).transpose(0, 1)
    ref = torch.from_numpy(g["y"])
    assert (y - ref).abs().max().item() < 1e-10


def test_text_transformer_eot_and_registry():
    torch.manual_seed(0)
    cls, _ = MODEL_REGISTRY.get("TextTransformer")
    assert cls is TextTransformer
    m = cls("TextTransformer", context_length=16, width=128, layers=2, vocab_size=100).double()
    text = torch.randint(1, 90, (4, 16))
    eot = torch.tensor([3, 15, 7, 0])
    text[torch.arange(4), eot] = 99  # end-of-text = largest id
    out = m(text, as_dict=True)["x"]
    assert out.shape == (4, 128)
    # causal: tokens after the end-of-text position do not change its feature
    t2 = text.clone()
    t2[0, 5:] = 1
    t2[0, 3] = 99
    assert torch.allclose(m(t2)[0], out[0])
    keys = set(m.state_dict())
    assert {"positional_embedding", "token_embedding.weight", "ln_final.weight",
            "transformer.resblocks.1.attn.in_proj_weight", "transformer.resblocks.1.mlp.c_proj.bias"} <= keys


def test_contrastive_head_and_loss_cpu_text():
    """MultiLabelContrastive's text half and TextContrastive (utils/loss.py:5-18)."""
    torch.manual_seed(1)
    text_cfg = EasyDict(name="TextTransformer", context_length=12, width=128, layers=1, vocab_size=64)
    tcls, _ = MODEL_REGISTRY.get("TextTransformer")
    tm = tcls(**text_cfg)
    text = torch.randint(1, 60, (3, 2, 12))
    text[..., -1] = 63
    feats = tm(text.view(-1, 12), as_dict=True)["x"].view(3, 2, -1)
    lin = torch.nn.Linear(128, 16)
    tf = lin(feats)
    pc = torch.randn(5, 16)
    has_text = torch.tensor([0, 2, 4])
    loss_fn, _ = LOSS_REGISTRY.get("TextContrastive")
    loss = loss_fn(pc, tf, has_text)
    sim = tf @ pc.T
    want = torch.nn.functional.cross_entropy(sim.transpose(1, 2), has_text[:, None].expand(3, 2))
    assert torch.allclose(loss, want)
    loss.backward()
    assert tm.token_embedding.weight.grad is not None


def test_tokenizer_matches_reference_fixture():
    """wsss3d.tokenizer restates the reference's CLIP BPE + fixed-shape text_transform
    (dataset/dataset_utils/tokenizer.py, text_transform_builder.py:33-76); token ids are bit-exact
    against ids the reference tokenizer produced (tests/golden/make_token_golden.py)."""
    import json
    import os
    from wsss3d.tokenizer import SimpleTokenizer, text_transform
    with open(os.path.join(os.path.dirname(__file__), "golden", "tokens.json")) as f:
        gold = json.load(f)
    tok = SimpleTokenizer()
    assert tok.encoder["<|startoftext|>"] == gold["specials"]["sot"]
    assert tok.encoder["<|endoftext|>"] == gold["specials"]["eot"]
    assert len(tok.encoder) == gold["specials"]["vocab"]
    for e in gold["encode"]:
        assert tok.encode(e["text"]) == e["ids"], e["text"]
    for c in gold["text_transform"]:
        ids = text_transform(c["max_seq_len"], c["cropped_texts"])(c["texts"])
        assert ids.dtype == torch.long
        assert ids.tolist() == c["ids"]
        # end-of-text is each row's largest id (TextTransformer reads the feature at argmax)
        assert (ids.argmax(-1) == (ids == gold["specials"]["eot"]).long().argmax(-1)).all()


def test_tokenizer_roundtrip_and_truncation():
    from wsss3d.tokenizer import Tokenize, default_tokenizer
    tok = default_tokenizer()
    text = "a grey office chair beside the desk"
    assert tok.decode(tok.encode(text)).strip() == text
    t = Tokenize(tok, 8)
    row = t("the sofa is in front of the television and the coffee table")
    assert row.shape == (8,) and row[0] == 49406 and row[-1] == 49407
    with pytest.raises(RuntimeError):
        Tokenize(tok, 8, truncate=False)(["the sofa is in front of the television and the coffee table"])
    assert Tokenize(tok, 8)([]).shape == (0, 8)
