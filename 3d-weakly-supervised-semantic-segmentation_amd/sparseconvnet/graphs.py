"""Capturing a training step into a HIP graph with a clean error path (an addition to the SCN API).

A step captured into `torch.cuda.CUDAGraph` (bench.py's graph loop, the reference's `train.py:69-81` step) that
raises inside the capture -- a library error (`MSP_REQUIRE`), a capacity check, an operation the capture refuses --
must not leave the capture open: torch's `~CUDAGraph` then fails with hipErrorStreamCaptureUnsupported and the
process ends in `std::terminate` (a core dump instead of the error; `profiles/r05/args_r05f_prefetch_gate_external_
event.log`).  `capture()` ends the capture and discards the graph before the error propagates, and undoes the
host-side state the discarded capture left behind:

* the metadata the capture consumed (`metadata.captured_metadata`): nothing will replay it;
* the step's weight images (`weight_images`): `prepare()` marked them fresh, but its split kernel was only captured,
  so the next step must not trust them;
* the caller's own state (`on_abort`, e.g. `wsss3d.dp.GradSync.abort`, which rejoins its exchange stream so the
  capture can end).

The process can then run the next step eagerly or capture it again (`tests/test_gpu_encoders.py::
test_capture_error_is_a_clean_error`).
"""
from __future__ import annotations

import torch

from . import metadata as _md
from . import weight_images as _wimg


def capture(body, stream, pool=None, mode="relaxed", on_abort=None):
    """Capture `body()` into a new graph on `stream`; returns (graph, body's result).  On an exception inside body
    the capture is ended, the graph discarded and the step's host state undone (module docstring), then the
    exception propagates unchanged."""
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        g.capture_begin(pool=pool, capture_error_mode=mode)
        try:
            out = body()
        except BaseException:
            abort(g, on_abort)
            raise
        g.capture_end()
    return g, out


def abort(g, on_abort=None):
    """End graph g's open capture (current stream = the capturing one) and discard it; see the module docstring."""
    if on_abort is not None:
        try:
            on_abort()  # first: streams that joined the capture rejoin it, or it cannot end
        except Exception:  # noqa: BLE001 -- the original error is the one to report
            pass
    try:
        g.capture_end()
    except Exception:  # noqa: BLE001 -- an invalidated capture: hipStreamEndCapture has ended it all the same
        pass
    try:
        g.reset()
    except Exception:  # noqa: BLE001
        pass
    _md.captured_metadata()
    wi = _wimg.active()
    if wi is not None:
        wi.invalidate()
