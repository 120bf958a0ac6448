"""Per-step split-weight images (an addition to the SCN API, optional; include/mi3dsparse.h msp_weight_image).

Every msp_conv_tile / msp_conv_local / msp_conv_nbr call splits its fp32 weights into an exact bf16-piece image
in its workspace -- one small launch per call, 116 per headline training step (0.6 ms of kernels plus their
launch gaps, `profiles/r03/step_kernels_r03s.txt`).  The weights change only at the optimizer step, so a training
loop can instead split every image the previous step used in ONE launch at the start of the step
(`prepare()`), and each convolution then finds its image ready (flip bit 2: the workspace already holds it).

    images = scn.weight_images.enable(model, optimizer=opt)   # the model's parameters own the cached weights
    for step ...:
        images.build()        # eagerly, outside any graph capture: allocate / upload what the last step added
        images.prepare()      # first thing of the step (may be inside a captured graph)
        ... forward, backward, optimizer ...

An image is used only when (1) `prepare()` launched its split after the weights last changed and (2) the call's
image descriptor is the recorded one; otherwise the call splits its own copy as before, and the new descriptor is
recorded for the next `build()`.  Changes are caught on the host, captures included: every optimizer step of the
optimizer given to `enable` (a step post-hook) and any in-place change that bumps a parameter's version counter
invalidate the images until the next `prepare()` -- torch's fused Adam does NOT bump version counters, hence the
hook (`tests/test_gpu_weight_images.py::test_stale_image_is_not_used`), which is why `enable` requires the
optimizer (`invalidate()` is public for weights changed any other way, e.g. `p.data` assignments or a
broadcast).  A parameter whose storage is replaced (`model.to()`, `p.data = ...`) drops its images at the next
`build()` / `prepare()`: no split ever reads a freed weight buffer.  Disabled (the default), nothing changes.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

_ACTIVE = None


class WeightImages:
    def __init__(self, params, device):
        self.device = torch.device(device)
        self.params = list(params)
        self.owners = {p.untyped_storage().data_ptr(): p for p in self.params}
        # key -> [desc, owner, img tensor or None, version at the last prepare or None, owner storage at record]
        self.entries = {}
        self.dirty = False
        self.table = None  # (descs device tensor, starts device tensor, n, total units)
        self.hits = 0      # calls that found their image prepared
        self._descs = {}   # (entry, n_rows, K, c_in, c_out, flip) -> descriptor template (or False)
        self.valid = False  # prepare() ran after the last optimizer step

    # ------------------------------------------------------------------ per call
    def _describe(self, entry, n_rows, K, c_in, c_out, flip):
        """msp_conv_weight_image for these arguments (memoised: a pure function of them)."""
        k = (entry, n_rows, K, c_in, c_out, flip)
        d = self._descs.get(k)
        if d is None:
            d = _lib.WeightImage()
            if _lib.load().msp_conv_weight_image(entry, n_rows, K, c_in, c_out, int(flip), ctypes.byref(d)):
                d = False
            if len(self._descs) > 1 << 14:
                self._descs.clear()
            self._descs[k] = d
        return d or None

    def lookup(self, entry, wt, n_rows, K, c_in, c_out, flip):
        """The prepared image tensor for this call, or None (the call then splits its own)."""
        owner = self.owners.get(wt.untyped_storage().data_ptr())
        if owner is None:
            return None
        d0 = self._describe(entry, n_rows, K, c_in, c_out, flip)
        if d0 is None:
            return None
        key = (wt.data_ptr(), tuple(wt.shape), d0.kind, d0.p, d0.wlay, d0.K, d0.c_in, d0.c_out)
        e = self.entries.get(key)
        if e is None:
            d = _lib.WeightImage.from_buffer_copy(d0)  # the entry's own descriptor (wt / img filled in)
            d.wt = wt.data_ptr()
            self.entries[key] = [d, owner, None, None, owner.untyped_storage().data_ptr()]
            self.dirty = True
            return None
        desc, _, img, version, _ = e
        if not self.valid or img is None or version is None or version != wt._version or img.numel() < d0.bytes:
            return None
        self.hits += 1
        return img

    # ------------------------------------------------------------------ per step
    def _prune(self):
        """Drop the images of parameters whose storage was replaced since they were recorded (their descriptors
        point at the old, possibly freed, buffer) and re-key the owners on the current storages."""
        stale = [k for k, e in self.entries.items() if e[1].untyped_storage().data_ptr() != e[4]]
        if stale:
            for k in stale:
                del self.entries[k]
            self.owners = {p.untyped_storage().data_ptr(): p for p in self.params}
            self.dirty = True
            self.table = None
            self.valid = False

    def build(self):
        """Allocate the images new descriptors need and upload the descriptor table (not inside a capture)."""
        self._prune()
        if not self.dirty or not self.entries:
            return
        if torch.cuda.is_current_stream_capturing():
            return
        descs, starts, total = [], [0], 0
        for e in self.entries.values():
            d = e[0]
            if e[2] is None:
                e[2] = torch.empty(max(int(d.bytes), 16), dtype=torch.uint8, device=self.device)
                d.img = e[2].data_ptr()
            descs.append(d)
            total += int(d.units)
            starts.append(total)
        arr = (_lib.WeightImage * len(descs))(*descs)
        raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        # blocking copies from pageable host memory (the host buffers are free to go when they return)
        self.table = (raw.to(self.device), torch.tensor(starts, dtype=torch.int64).to(self.device), len(descs), total)
        self.dirty = False

    def prepare(self):
        """Split every recorded image in one launch on the current stream (capturable).  Returns whether it ran."""
        self._prune()
        if self.dirty:
            self.build()
        if self.table is None or self.dirty:
            return False
        descs, starts, n, total = self.table
        _lib.call("msp_split_weight_images", _lib.ptr(descs), n, _lib.ptr(starts), total, _lib.stream(self.device))
        for e in self.entries.values():
            e[3] = e[1]._version
        self.valid = True
        return True

    def invalidate(self, *args, **kwargs):
        """The weights changed (optimizer step post-hook): no image is used until the next prepare()."""
        self.valid = False


def enable(model, device=None, optimizer=None):
    """Turn per-step images on for the parameters of `model` (returns the manager).  `optimizer` (required): the
    optimizer that updates these parameters -- its steps invalidate the images.  Fused / capturable optimizers
    do not bump parameter version counters, so without the hook a stale image would go unnoticed."""
    global _ACTIVE
    if optimizer is None or not hasattr(optimizer, "register_step_post_hook"):
        raise ValueError("sparseconvnet.weight_images.enable: pass the optimizer that updates the model's parameters "
                         "(its step post-hook invalidates the images)")
    params = list(model.parameters())
    dev = device if device is not None else (params[0].device if params else "cuda")
    _ACTIVE = WeightImages(params, dev)
    optimizer.register_step_post_hook(_ACTIVE.invalidate)
    return _ACTIVE


def disable():
    global _ACTIVE
    _ACTIVE = None


def active():
    return _ACTIVE
