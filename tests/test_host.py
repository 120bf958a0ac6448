"""Host-side logic on CPU: registry, encoder topology against the reference's
own model file (tests/golden/topology.json), EasyDict, checkpoints, the
synthetic batch producer, heads and losses.  No GPU compute."""
import json
import os

import numpy as np
import pytest
import torch

import sparseconvnet as scn
from oracle.encoders import OracleEncoder
from wsss3d import EasyDict, LOSS_REGISTRY, MODEL_REGISTRY, Registry, segment_mean
from wsss3d.synthetic import make_batch, make_room, train_merge, val_merge

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_registry_semantics():
    r = Registry("t")

    @r.register(embed_length=lambda m: 2 * m)
    class A:
        pass

    assert r.get("A")[0] is A and r.get("A")[1]["embed_length"](3) == 6
    with pytest.raises(AssertionError):
        r.register(A)
    r.register(type("B", (), {}), suffix="3d")
    assert r.get("B")[0].__name__ == "B"  # falls back to B_3d
    with pytest.raises(KeyError):
        r.get("nope")
    assert "A" in r and set(r.keys()) == {"A", "B_3d"}


@pytest.mark.parametrize("key", json.load(open(os.path.join(GOLD, "topology.json"))).keys())
def test_topology_matches_reference_model_file(key):
    """state_dict keys/shapes, parameter count and embed_length of every
    encoder equal those of the reference's models/SparseConvNet.py."""
    want = json.load(open(os.path.join(GOLD, "topology.json")))[key]
    name, m, r, res = key.split("-")
    cls, meta = MODEL_REGISTRY.get(name)
    enc = cls(name, m=int(m[1:]), dimension=3, full_scale=4096, block_reps=int(r[1:]), residual_blocks=bool(int(res)))
    got = [[k, list(v.shape)] for k, v in enc.state_dict().items()]
    assert got == want["state_dict"]
    assert sum(p.numel() for p in enc.parameters()) == want["n_params"]
    assert meta["embed_length"](int(m[1:])) == want["embed_length"]


@pytest.mark.parametrize("name,m,reps,res,params", [
    ("SparseConvFCNetEncoder", 16, 1, False, 1_200_144),   # C1
    ("SparseConvUNet", 16, 1, False, 2_689_520),           # C2
    ("SparseConvUNet", 32, 2, True, 30_103_712),           # C3 / C4 (headline)
    ("SparseConvFCNet", 32, 1, False, 4_795_744),          # C5
])
def test_baseline_config_sizes(name, m, reps, res, params):
    cls, _ = MODEL_REGISTRY.get(name)
    enc = cls(name, m=m, dimension=3, full_scale=4096, block_reps=reps, residual_blocks=res)
    assert sum(p.numel() for p in enc.parameters()) == params


@pytest.mark.parametrize("name,m,reps,res", [("SparseConvUNet", 32, 2, True), ("SparseConvFCNet", 16, 1, False),
                                             ("SparseConvFCNetDirectUpPoolLight", 16, 1, True),
                                             ("SparseConvFCNetEncoder", 16, 1, False)])
def test_seeded_init_equals_oracle(name, m, reps, res):
    """Same module tree and same RNG draw order as the oracle (and SCN's
    builders): a seeded construction gives bit-identical weights."""
    torch.manual_seed(11)
    a = MODEL_REGISTRY.get(name)[0](name, m=m, dimension=3, full_scale=4096, block_reps=reps, residual_blocks=res)
    torch.manual_seed(11)
    b = OracleEncoder(name, m=m, block_reps=reps, residual_blocks=res)
    sa, sb = a.state_dict(), b.state_dict()
    assert list(sa) == list(sb) and all(torch.equal(sa[k], sb[k]) for k in sa)


def test_encoder_name_and_input_checks():
    cls, _ = MODEL_REGISTRY.get("SparseConvUNet")
    with pytest.raises(AssertionError):
        cls("SparseConvFCNet", m=16, dimension=3, full_scale=4096, block_reps=1, residual_blocks=False)
    enc = cls("SparseConvUNet", m=16, dimension=3, full_scale=4096, block_reps=1, residual_blocks=False)
    with pytest.raises(AssertionError):
        enc([torch.zeros(3, 4), torch.zeros(3, 3)])
    with pytest.raises(AssertionError):
        enc(EasyDict(coords=torch.zeros(3, 4), feature=torch.zeros(2, 3), batch_offsets=[0, 3]))


def test_module_api_limits():
    with pytest.raises(NotImplementedError):
        scn.SubmanifoldConvolution(3, 4, 4, 3, False, groups=2)
    with pytest.raises(NotImplementedError):
        scn.Convolution(3, 4, 4, 3, 2, False)
    with pytest.raises(NotImplementedError):
        scn.InputLayer(2, 16)
    w = scn.SubmanifoldConvolution(3, 8, 4, 3, False).weight
    assert w.shape == (27, 1, 8, 4) and abs(w.std().item() - (2 / 8 / 27) ** 0.5) < 0.05
    bn = scn.BatchNormReLU(5)
    assert bn.eps == 1e-4 and bn.momentum == 0.9 and bn.leakiness == 0
    assert set(bn.state_dict()) == {"weight", "bias", "running_mean", "running_var"}


def test_feature_path_refuses_cpu_tensors():
    """No CPU fallback: the product raises on host tensors."""
    inp = scn.InputLayer(3, 16, mode=4)
    with pytest.raises(RuntimeError):
        inp([torch.zeros(2, 4, dtype=torch.long), torch.zeros(2, 3)])


def test_easydict():
    d = EasyDict(a=1, b={"c": 2, "d": [{"e": 3}]})
    assert d.a == 1 and d.b.c == 2 and d.b.d[0].e == 3
    d.f = {"g": 4}
    assert d["f"].g == 4 and isinstance(d, dict)


def test_checkpoint_naming_and_pruning(tmp_path):
    model = torch.nn.Linear(3, 2)
    exp = str(tmp_path / "run" / "run")
    os.makedirs(os.path.dirname(exp))
    assert scn.checkpoint_restore(model, exp, "model", use_cuda=False) == 1
    for e in range(1, 7):
        scn.checkpoint_save(model, exp, "model", e, use_cuda=False)
    kept = sorted(os.listdir(tmp_path / "run"))
    assert kept == [f"run-{e:09d}-model.pth" for e in (1, 2, 4, 6)]
    with torch.no_grad():
        model.weight.zero_()
    assert scn.checkpoint_restore(model, exp, "model", use_cuda=False) == 7
    assert model.weight.abs().sum() > 0
    assert scn.is_power2(64) and not scn.is_power2(96) and not scn.is_power2(0)


def test_synthetic_batch_contract():
    b = make_batch(2, 20, seed=3, spacing=0.1)
    c = b["coords"]
    assert c.dtype == np.int64 and c.shape[1] == 4
    assert c[:, :3].min() >= 0 and c[:, :3].max() < 4096
    assert set(np.unique(c[:, 3])) == {0, 1}
    off = b["batch_offsets"]
    assert off[0] == 0 and off[-1] == len(c) and all(np.all(c[off[i]:off[i + 1], 3] == i) for i in range(2))
    assert b["feats"].shape == (len(c), 3) and b["scene_labels"].shape == (2, 20)
    b2 = make_batch(2, 20, seed=3, spacing=0.1)
    assert np.array_equal(b2["coords"], c) and np.array_equal(b2["feats"], b["feats"])
    room = make_room(0, spacing=0.1)
    v = val_merge([room], 20)
    assert v["coords"].shape[0] == v["feats"].shape[0] == v["point_ids"].shape[0]
    t = train_merge([room, room], 50)
    assert t["batch_offsets"][1] <= len(room[0])


def test_segment_mean_and_losses():
    f = torch.arange(12.0).view(6, 2)
    assert torch.equal(segment_mean(f, [0, 2, 6]), torch.tensor([[1.0, 2.0], [7.0, 8.0]]))
    cls_loss, _ = LOSS_REGISTRY.get("Classification")
    logits = torch.randn(4, 20)
    y = (torch.rand(4, 20) > 0.5).float()
    assert torch.allclose(cls_loss(logits, y), torch.nn.functional.multilabel_soft_margin_loss(logits, y))
    pl = torch.tensor([1, -100, 3, 4])
    ref = torch.nn.functional.cross_entropy(logits[[0, 2, 3]], pl[[0, 2, 3]])
    assert torch.allclose(cls_loss(logits, pl), ref)
    tc, _ = LOSS_REGISTRY.get("TextContrastive")
    assert tc(torch.randn(2, 8), torch.randn(1, 3, 8), torch.tensor([], dtype=torch.long)) == 0
    val = tc(torch.randn(2, 8), torch.randn(2, 3, 8), torch.tensor([0, 1]))
    assert val.ndim == 0 and torch.isfinite(val)


def test_balanced_shards():
    from wsss3d.dp import balanced_shards
    sizes = [100, 90, 80, 10, 20, 30, 40, 50, 60]
    sh = balanced_shards(sizes, 2)
    assert [len(s) for s in sh] == [4, 4]
    assert len(set(sh[0]) | set(sh[1])) == 8 and 3 not in sh[0] + sh[1]  # smallest scene dropped
    loads = [sum(sizes[i] for i in s) for s in sh]
    assert abs(loads[0] - loads[1]) <= 20


REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present (GPU box)")
def test_reference_model_file_runs_on_this_package():
    """Drop-in check: the reference's models/SparseConvNet.py, loaded unmodified
    with THIS package as `sparseconvnet`, registers its encoders and builds
    module trees identical (keys, shapes, seeded values) to wsss3d's."""
    import importlib.util
    import sys
    import types
    sys.modules["easydict"] = types.SimpleNamespace(EasyDict=EasyDict)
    if REF not in sys.path:
        sys.path.append(REF)
    spec = importlib.util.spec_from_file_location("ref_models_on_mi3dsparse", os.path.join(REF, "models", "SparseConvNet.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.scn is scn
    for name, m, reps, res in [("SparseConvUNet", 32, 2, True), ("SparseConvFCNet", 16, 1, False),
                               ("SparseConvFCNetDirectUpPoolLight", 16, 1, True)]:
        torch.manual_seed(5)
        ref_enc = getattr(mod, name)(name, m=m, dimension=3, full_scale=4096, block_reps=reps, residual_blocks=res)
        torch.manual_seed(5)
        ours = MODEL_REGISTRY.get(name)[0](name, m=m, dimension=3, full_scale=4096, block_reps=reps,
                                           residual_blocks=res)
        a, b = ref_enc.state_dict(), ours.state_dict()
        assert list(a) == list(b) and all(torch.equal(a[k], b[k]) for k in a), name


def test_scene_ranges_match_host_logic():
    """The fused tail's validity check (InputRules.scene_ranges_match): scene b of batch_offsets must be
    exactly the points of batch id b, decided from the scene starts read back with the voxel count."""
    from sparseconvnet.metadata import InputRules
    r = InputRules(10, None, None, None, 3)
    r.batch_monotonic, r.scene_starts = True, [0, 4, 4, 10]     # ids 0..2, id 1 empty
    assert r.scene_ranges_match([0, 4, 4, 10])
    assert r.scene_ranges_match([0, 4, 4, 10, 10])              # a trailing empty scene
    assert not r.scene_ranges_match([0, 3, 4, 10])
    assert not r.scene_ranges_match([0, 4, 10])                 # fewer scenes than batch ids
    assert not r.scene_ranges_match([0, 10])
    r.batch_monotonic = False
    assert not r.scene_ranges_match([0, 4, 4, 10])
    r.batch_monotonic, r.scene_starts = True, None
    assert not r.scene_ranges_match([0, 4, 4, 10])


def test_bench_presets_and_host_cores():
    import bench
    assert bench.PRESETS["c3"]["batch"] == 8 and bench.PRESETS["c4"]["batch"] == 5
    assert bench.PRESETS["c2"]["m"] == 16 and bench.PRESETS["c2"]["residual"] == 0
    cores, info = bench.host_cores()
    assert 1 <= cores <= (os.cpu_count() or cores) and info["cpu_model"]
    assert bench.family("subm_fwd/x6g") == "conv" and bench.family("wgrad/x6") == "wgrad"
    assert bench.family("bn_fwd/hbm") == "bn" and bench.family("deconv_fwd/f32") == "pairs"
