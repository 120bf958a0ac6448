"""Device batch assembly (wsss3d/merge.py, msp_merge) against the numpy
restatement of trainMerge / valMerge (wsss3d/synthetic.py,
dataset/data.py:135-238, 256-310) on the same scenes and random draws:
integer outputs bit-exact, colours exact (same f32 add)."""
import numpy as np
import pytest
import torch

from wsss3d.merge import DeviceScenes, train_merge_gpu, val_merge_gpu
from wsss3d.synthetic import make_room, train_merge, val_merge

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,scale,seed", [(3, 50, 0), (2, 20, 5), (1, 50, 9)])
def test_train_merge_gpu_bitexact(n, scale, seed):
    scenes = [make_room(100 + seed * 10 + i, spacing=0.03) for i in range(n)]
    ref = train_merge(scenes, scale, seed=seed)
    got = train_merge_gpu(DeviceScenes(scenes), scale, seed=seed)
    assert got.x.batch_offsets == ref["batch_offsets"]
    assert np.array_equal(got.x.coords.cpu().numpy(), ref["coords"])
    assert np.array_equal(got.x.feature.cpu().numpy(), ref["feats"])
    assert np.array_equal(got.y_orig.cpu().numpy(), ref["labels"])
    assert np.array_equal(got.y.cpu().numpy(), ref["scene_labels"])


def test_train_merge_gpu_crops():
    """A scene larger than full_scale: the crop (data.py:181) drops points."""
    scenes = [make_room(7, spacing=0.05)]
    ref = train_merge(scenes, 400, full_scale=1024, seed=1)
    got = train_merge_gpu(DeviceScenes(scenes), 400, full_scale=1024, seed=1)
    assert ref["batch_offsets"][-1] < len(scenes[0][0])
    assert got.x.batch_offsets == ref["batch_offsets"]
    assert np.array_equal(got.x.coords.cpu().numpy(), ref["coords"])


def test_val_merge_gpu_bitexact():
    scenes = [make_room(300 + i, spacing=0.03) for i in range(3)]
    ref = val_merge(scenes, 50, seed=2)
    got = val_merge_gpu(DeviceScenes(scenes), 50, seed=2)
    assert np.array_equal(got.x.coords.cpu().numpy(), ref["coords"])
    assert np.array_equal(got.x.feature.cpu().numpy(), ref["feats"])
    assert np.array_equal(got.y_orig.cpu().numpy(), ref["labels"])
    assert np.array_equal(got.point_ids.cpu().numpy(), ref["point_ids"])
