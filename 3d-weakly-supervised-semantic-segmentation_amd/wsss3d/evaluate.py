"""Validation accumulation on the device (train.py:94-116).

The reference's eval loop is

    store = torch.zeros(valOffsets[-1], 20)
    for rep in range(1, 1 + val_reps):
        for batch in val_data_loader:
            predictions = model(batch['x'])                              # (N, 20) per-point logits
            store.index_add_(0, batch['point_ids'], predictions.cpu())   # train.py:107
    mean_iou = iou.evaluate(store.max(1)[1].numpy(), valLabels)

`PointLogitStore` keeps `store` in HBM: `add()` is the `index_add_` on the device (msp_index_add_rows,
bit-equal to the CPU loop for any ids, repeated ids included), so the per-batch device-to-host copy of
the (N, 20) predictions goes away; `cpu()` / `argmax()` hand the result to the reference's
`utils/iou.py` once per evaluation.  The predictions come from the heads' fused eval path
(heads.point_logits: the Linear on the voxel rows, no (N, C) feature tensor).
"""
from __future__ import annotations

import torch

from sparseconvnet.ops import index_add_rows

from .synthetic import NUM_CLASSES


class PointLogitStore:
    """Device twin of train.py:96's `store = torch.zeros(valOffsets[-1], 20)`."""

    def __init__(self, n_points: int, device, n_classes: int = NUM_CLASSES):
        self.store = torch.zeros((int(n_points), int(n_classes)), dtype=torch.float32, device=device)

    def add(self, point_ids: torch.Tensor, predictions: torch.Tensor):
        """store.index_add_(0, point_ids, predictions) (train.py:107)."""
        index_add_rows(self.store, point_ids, predictions.detach())
        return self

    def argmax(self) -> torch.Tensor:
        """store.max(1)[1] (train.py:114)."""
        return self.store.max(1)[1]

    def cpu(self) -> torch.Tensor:
        return self.store.cpu()
