"""Batch assembly on the device.

`trainMerge` / `valMerge` (`dataset/data.py:135-238, 256-310`) run per batch
in the reference's DataLoader workers on the CPU; once the encoder step is on
the GPU that collation becomes the bottleneck.  Here the raw scenes stay in
HBM and `msp_merge` does the per-point work (rotation/scale, random offset,
crop, `.long()`, batch column, colour shift, scene labels, batch offsets) in
one pass; only the data-independent random draws come from the host, drawn
exactly as the numpy restatement (`wsss3d/synthetic.py: train_params,
val_params`) draws them, so both paths produce the same batch.
"""
from __future__ import annotations

import numpy as np
import torch

from sparseconvnet import _lib
from sparseconvnet._lib import call, ptr

from .edict import EasyDict
from .synthetic import NUM_CLASSES, train_params, val_params


class DeviceScenes:
    """Raw scenes resident in HBM: concatenated xyz / rgb (f32) and labels
    (int64), with the per-scene point ranges."""

    def __init__(self, scenes, device="cuda"):
        sizes = [len(a) for a, _, _ in scenes]
        self.start = [0]
        for n in sizes:
            self.start.append(self.start[-1] + n)
        self.max_points = max(sizes) if sizes else 0
        dev = torch.device(device)
        self.xyz = torch.from_numpy(np.concatenate([a for a, _, _ in scenes]).astype(np.float32)).to(dev)
        self.rgb = torch.from_numpy(np.concatenate([b for _, b, _ in scenes]).astype(np.float32)).to(dev)
        self.labels = torch.from_numpy(np.concatenate([c for _, _, c in scenes]).astype(np.int64)).to(dev)
        self.start_dev = torch.tensor(self.start, dtype=torch.int64, device=dev)
        self.device = dev

    def __len__(self):
        return len(self.start) - 1


def _merge(sc: DeviceScenes, params, mode, full_scale, point_id_base=0):
    B = len(sc)
    dev = sc.device
    rot = torch.tensor(np.stack([p[0] for p in params]).reshape(B, 9), dtype=torch.float64, device=dev)
    c1 = torch.tensor(np.stack([p[1] for p in params]), dtype=torch.float64, device=dev)
    c2 = torch.tensor(np.stack([p[2] for p in params]), dtype=torch.float64, device=dev)
    u1 = torch.tensor(np.stack([p[3] for p in params]), dtype=torch.float64, device=dev)
    u2 = torch.tensor(np.stack([p[4] for p in params]), dtype=torch.float64, device=dev)
    shift = torch.tensor(np.stack([p[5] for p in params]), dtype=torch.float32, device=dev)
    P = sc.start[-1]
    coords = torch.empty((max(P, 1), 4), dtype=torch.int64, device=dev)
    feats = torch.empty((max(P, 1), 3), dtype=torch.float32, device=dev)
    labels = torch.empty(max(P, 1), dtype=torch.int64, device=dev)
    ids = torch.empty(max(P, 1), dtype=torch.int64, device=dev) if mode == 1 else None
    offsets = torch.empty(B + 1, dtype=torch.int64, device=dev)
    scene_labels = torch.empty((B, NUM_CLASSES), dtype=torch.float32, device=dev)
    wsb = int(_lib.query("msp_merge_workspace_size", B, _lib.I64(sc.max_points)))
    ws = torch.empty(max(wsb, 8), dtype=torch.uint8, device=dev)
    call("msp_merge", ptr(sc.xyz), ptr(sc.rgb), ptr(sc.labels), ptr(sc.start_dev), B, sc.max_points, mode,
         float(full_scale), ptr(rot), ptr(c1), ptr(c2), ptr(u1), ptr(u2), ptr(shift), NUM_CLASSES, ptr(coords),
         ptr(feats), ptr(labels), ptr(ids), int(point_id_base), ptr(offsets), ptr(scene_labels), ptr(ws), wsb,
         _lib.stream(dev))
    off = offsets.tolist()  # the one host read: batch_offsets is a python list in the reference
    n = off[-1]
    return coords[:n], feats[:n], labels[:n], (ids[:n] if ids is not None else None), off, scene_labels


def train_merge_gpu(sc: DeviceScenes, scale: float, full_scale: int = 4096, seed: int = 0):
    """Device `trainMerge`: EasyDict(x=EasyDict(coords, feature, batch_offsets),
    y_orig, y) like the reference's batch (`dataset/data.py:224-238`, point-cloud
    part); bitwise equal to wsss3d.synthetic.train_merge on the same scenes."""
    params = [train_params(scale, seed, i) for i in range(len(sc))]
    coords, feats, labels, _, off, sl = _merge(sc, params, 0, full_scale)
    return EasyDict(x=EasyDict(coords=coords, feature=feats, batch_offsets=off), y_orig=labels, y=sl)


def val_merge_gpu(sc: DeviceScenes, scale: float, full_scale: int = 4096, seed: int = 0, point_id_base=0):
    """Device `valMerge` (`dataset/data.py:256-310`): coords, feats, labels and
    the ids of the kept points (offset by point_id_base, the reference's
    valOffsets[i] for the first scene)."""
    params = []
    for i in range(len(sc)):
        m, _, c2, u1, u2, shift = val_params(scale, seed, i)
        params.append((m, np.full(3, full_scale / 2), c2, u1, u2, shift))
    coords, feats, labels, ids, off, sl = _merge(sc, params, 1, full_scale, point_id_base)
    return EasyDict(x=EasyDict(coords=coords, feature=feats), y_orig=labels, y=sl.long(), point_ids=ids,
                    batch_offsets=off)
