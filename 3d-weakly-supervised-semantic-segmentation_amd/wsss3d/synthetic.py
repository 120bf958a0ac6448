"""Synthetic ScanNet-shaped scenes and the reference's batch transform.

The reference trains on preprocessed ScanNet v2 scenes that are not in this
container (`dataset/data.py:89-130` loads them at import time).  This module
produces scenes with the same value distribution:

* procedural rooms: floor + 4 walls + 6-10 box furniture, W, D ~ U(3.5, 5.5) m,
  H ~ U(2.4, 2.8) m, surfaces sampled uniformly at ~2 cm spacing (~2e5 points),
  Gaussian jitter sigma = 5 mm, coordinates centred like
  `dataset/ScanNet/prepare_data.py:29-30`;
* colours in [-1, 1] (`prepare_data.py:31`), piecewise constant per surface
  + N(0, 0.05); labels in 0..19 with ~5 % ignored (-100).

`train_merge` restates the geometric part of `trainMerge`
(`dataset/data.py:135-238`): random scale/flip/rotation, random offset into
[0, full_scale)^3, crop, `.long()` truncation, batch id in the LAST column
(`:198`), per-scene colour shift N(0, 0.1) (`:200`) and the cumulative
`batch_offsets` list (`:142,209`).  `val_merge` restates `valMerge`
(`:256-310`).  Randomness is numpy-seeded so every consumer (oracle, GPU
tests, bench) sees identical inputs.
"""
from __future__ import annotations

import numpy as np

NUM_CLASSES = 20  # dataset/data.py:7


def _sample_rect(rng, origin, u, v, spacing):
    """Uniform random samples on the parallelogram origin + a*u + b*v."""
    area = np.linalg.norm(np.cross(u, v))
    n = max(1, int(round(area / (spacing * spacing))))
    ab = rng.random((n, 2))
    return origin[None, :] + ab[:, :1] * u[None, :] + ab[:, 1:] * v[None, :]


def make_room(seed: int, spacing: float = 0.02, jitter: float = 0.005):
    """One procedural room.  Returns (coords f32 (N,3) metres, colours f32 (N,3) in
    [-1,1], labels int64 (N,))."""
    rng = np.random.default_rng(seed)
    W, D, H = rng.uniform(3.5, 5.5), rng.uniform(3.5, 5.5), rng.uniform(2.4, 2.8)
    surfaces = []  # (points, label)
    ex, ey, ez = np.eye(3)
    surfaces.append((_sample_rect(rng, np.zeros(3), W * ex, D * ey, spacing), 1))  # floor
    surfaces.append((_sample_rect(rng, np.zeros(3), W * ex, H * ez, spacing), 0))  # walls
    surfaces.append((_sample_rect(rng, D * ey, W * ex, H * ez, spacing), 0))
    surfaces.append((_sample_rect(rng, np.zeros(3), D * ey, H * ez, spacing), 0))
    surfaces.append((_sample_rect(rng, W * ex, D * ey, H * ez, spacing), 0))
    for _ in range(int(rng.integers(6, 11))):
        sx, sy, sz = rng.uniform(0.3, 1.6), rng.uniform(0.3, 1.2), rng.uniform(0.4, 1.2)
        x0, y0 = rng.uniform(0.05, W - sx - 0.05), rng.uniform(0.05, D - sy - 0.05)
        o = np.array([x0, y0, 0.0])
        lab = int(rng.integers(2, NUM_CLASSES))
        surfaces.append((_sample_rect(rng, o + sz * ez, sx * ex, sy * ey, spacing), lab))  # top
        surfaces.append((_sample_rect(rng, o, sx * ex, sz * ez, spacing), lab))
        surfaces.append((_sample_rect(rng, o + sy * ey, sx * ex, sz * ez, spacing), lab))
        surfaces.append((_sample_rect(rng, o, sy * ey, sz * ez, spacing), lab))
        surfaces.append((_sample_rect(rng, o + sx * ex, sy * ey, sz * ez, spacing), lab))
    pts, cols, labs = [], [], []
    for p, lab in surfaces:
        base = rng.uniform(-0.8, 0.8, 3)
        pts.append(p)
        cols.append(np.clip(base[None, :] + rng.normal(0, 0.05, (len(p), 3)), -1, 1))
        labs.append(np.full(len(p), lab, np.int64))
    coords = np.concatenate(pts, 0)
    coords += rng.normal(0, jitter, coords.shape)
    coords -= coords.mean(0)  # prepare_data.py:29-30 centring
    colours = np.concatenate(cols, 0)
    labels = np.concatenate(labs, 0)
    labels[rng.random(len(labels)) < 0.05] = -100
    return coords.astype(np.float32), colours.astype(np.float32), labels


def train_params(scale: float, seed: int, idx: int):
    """The random draws of `trainMerge` for scene idx (`dataset/data.py:165-178, 200`),
    in the reference's order: jitter matrix, flip, rotation angle, the two
    rand(3) of the offset, the colour shift.  They do not depend on the data,
    so the device batch assembly (wsss3d/merge.py) uses the same draws.
    Returns (rot (3,3) f64, c1 (3,), c2 (3,), u1 (3,), u2 (3,), shift (3,) f32)."""
    rng = np.random.RandomState(1000 + seed * 997 + idx)
    m = np.eye(3) + rng.randn(3, 3) * 0.1  # data.py:165
    m[0][0] *= rng.randint(0, 2) * 2 - 1
    m *= scale
    theta = rng.rand() * 2 * np.pi
    rot = np.matmul(m, [[np.cos(theta), np.sin(theta), 0], [-np.sin(theta), np.cos(theta), 0], [0, 0, 1]])
    u1, u2 = rng.rand(3), rng.rand(3)  # data.py:178, left to right
    shift = rng.randn(3).astype(np.float32) * 0.1  # data.py:200
    return rot, np.zeros(3), np.zeros(3), u1, u2, shift


def val_params(scale: float, seed: int, idx: int):
    """The random draws of `valMerge` (`dataset/data.py:263-275`): flip,
    rotation, the centring jitter U(-2, 2)^3, the two rand(3) of the offset."""
    rng = np.random.RandomState(2000 + seed * 997 + idx)
    m = np.eye(3)
    m[0][0] *= rng.randint(0, 2) * 2 - 1
    m *= scale
    theta = rng.rand() * 2 * np.pi
    m = np.matmul(m, [[np.cos(theta), np.sin(theta), 0], [-np.sin(theta), np.cos(theta), 0], [0, 0, 1]])
    c2 = rng.uniform(-2, 2, 3)
    u1, u2 = rng.rand(3), rng.rand(3)
    return m, None, c2, u1, u2, np.zeros(3, np.float32)


def transform(a, rot, c1, c2):
    """a . rot + c1 + c2 in fp64, each product and sum rounded in a fixed order
    ((a0 r0j + a1 r1j) + a2 r2j) + c1j + c2j -- the reference's np.matmul in
    float64 up to BLAS summation order; the device path uses the same order."""
    a = a.astype(np.float64)
    t = (a[:, 0:1] * rot[0][None, :] + a[:, 1:2] * rot[1][None, :]) + a[:, 2:3] * rot[2][None, :]
    return (t + c1[None, :]) + c2[None, :]


def _place(t, u1, u2, full_scale, mode):
    """Random offset into [0, full_scale)^3 and the crop (data.py:174-182 train,
    :271-277 val; each formula in its own evaluation order)."""
    lo, hi = t.min(0), t.max(0)
    if mode == "train":
        length = hi - lo
        q1, q2 = full_scale - length - 0.001, full_scale - length + 0.001
    else:
        q1, q2 = full_scale - hi + lo - 0.001, full_scale - hi + lo + 0.001
    offset = -lo + np.clip(q1, 0, None) * u1 + np.clip(q2, None, 0) * u2
    p = t + offset
    keep = (p.min(1) >= 0) * (p.max(1) < full_scale)
    return p, keep


def train_merge(scenes, scale: float, full_scale: int = 4096, seed: int = 0):
    """Restates `trainMerge` (`dataset/data.py:135-238`) for the point-cloud part.

    Returns dict(coords int64 (N,4) [x,y,z,b], feats f32 (N,3),
    batch_offsets list[int], labels int64 (N,), scene_labels f32 (B,20)).
    """
    locs, feats, labels, scene_labels = [], [], [], []
    batch_offsets = [0]
    for idx, (a, b, c) in enumerate(scenes):
        rot, c1, c2, u1, u2, shift = train_params(scale, seed, idx)
        p, keep = _place(transform(a, rot, c1, c2), u1, u2, full_scale, "train")
        a, bb, cc = p[keep], b[keep], c[keep]
        a = a.astype(np.int64)  # torch.from_numpy(a).long() truncates toward zero
        sl = np.zeros(NUM_CLASSES, np.float32)
        u = np.unique(cc)
        sl[u[u >= 0]] = 1.0
        locs.append(np.concatenate([a, np.full((len(a), 1), idx, np.int64)], 1))
        feats.append(bb + shift)  # data.py:200
        labels.append(cc)
        scene_labels.append(sl)
        batch_offsets.append(batch_offsets[-1] + int(keep.sum()))
    return dict(coords=np.concatenate(locs, 0), feats=np.concatenate(feats, 0).astype(np.float32),
                batch_offsets=batch_offsets, labels=np.concatenate(labels, 0),
                scene_labels=np.stack(scene_labels, 0))


def val_merge(scenes, scale: float, full_scale: int = 4096, seed: int = 0):
    """Restates `valMerge` (`dataset/data.py:256-310`): no jitter of the matrix,
    centre at full_scale/2 + U(-2, 2), same crop and `.long()`."""
    locs, feats, labels, point_ids = [], [], [], []
    base = 0
    for idx, (a, b, c) in enumerate(scenes):
        m, _, c2, u1, u2, _ = val_params(scale, seed, idx)
        p, keep = _place(transform(a, m, np.full(3, full_scale / 2), c2), u1, u2, full_scale, "val")
        a = p[keep].astype(np.int64)
        locs.append(np.concatenate([a, np.full((len(a), 1), idx, np.int64)], 1))
        feats.append(b[keep])
        labels.append(c[keep])
        point_ids.append(np.nonzero(keep)[0] + base)
        base += len(keep)
    return dict(coords=np.concatenate(locs, 0), feats=np.concatenate(feats, 0).astype(np.float32),
                labels=np.concatenate(labels, 0), point_ids=np.concatenate(point_ids, 0))


def make_batch(n_scenes: int, scale: float, seed: int = 0, full_scale: int = 4096,
               spacing: float = 0.02):
    """n_scenes procedural rooms pushed through `train_merge`."""
    scenes = [make_room(seed * 1000 + i, spacing=spacing) for i in range(n_scenes)]
    return train_merge(scenes, scale, full_scale, seed)


def random_cloud(n_points: int, extent: int, n_batch: int = 1, seed: int = 0,
                 n_feat: int = 3, dense_frac: float = 0.0):
    """Small random clouds for op-level tests: integer coords in [0, extent)^3
    with duplicates (so mode-4 averaging is exercised)."""
    rng = np.random.default_rng(seed)
    coords = rng.integers(0, extent, (n_points, 3))
    if dense_frac > 0:  # force duplicates
        k = int(n_points * dense_frac)
        coords[:k] = coords[rng.integers(0, n_points, k)]
    b = rng.integers(0, n_batch, (n_points, 1))
    feats = rng.standard_normal((n_points, n_feat)).astype(np.float32)
    return np.concatenate([coords, b], 1).astype(np.int64), feats
