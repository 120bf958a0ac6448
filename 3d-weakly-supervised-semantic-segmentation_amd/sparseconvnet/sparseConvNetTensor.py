"""SparseConvNetTensor: features of the active sites + the shared metadata."""
from __future__ import annotations

import torch


class SparseConvNetTensor(object):
    """Same fields as SCN's tensor: `features` (V, C) float32 on the device,
    `metadata` (shared by every layer of one forward) and `spatial_size`
    (LongTensor of the per-axis size)."""

    def __init__(self, features=None, metadata=None, spatial_size=None):
        self.features = features
        self.metadata = metadata
        if spatial_size is not None and not torch.is_tensor(spatial_size):
            spatial_size = torch.LongTensor(list(spatial_size))
        self.spatial_size = spatial_size

    @property
    def size_int(self) -> int:
        return int(self.spatial_size[0])

    def get_spatial_locations(self, spatial_size=None):
        """(V, 4) int64 [x, y, z, batch] of the active sites, row-aligned with
        `features`."""
        size = self.size_int if spatial_size is None else int(torch.as_tensor(spatial_size).view(-1)[0])
        return self.metadata.locations(size)

    def batch_size(self):
        return self.metadata.input.batch_size

    def cuda(self):
        self.features = self.features.cuda()
        return self

    def to(self, *args, **kw):
        self.features = self.features.to(*args, **kw)
        return self

    def detach(self):
        return SparseConvNetTensor(self.features.detach(), self.metadata, self.spatial_size)

    def __repr__(self):
        f = None if self.features is None else tuple(self.features.shape)
        s = None if self.spatial_size is None else self.spatial_size.tolist()
        return f"SparseConvNetTensor<features={f}, spatial_size={s}>"
