"""ctypes binding of libmi3dsparse.so (the C ABI in include/mi3dsparse.h).

The library is the only compute path: there is no CPU or eager-PyTorch
fallback.  If the .so is missing, or a tensor handed to it is not a HIP
device tensor, the call raises instead of silently running elsewhere.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_double, c_float, c_int, c_int64, c_size_t, c_void_p

import torch

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MI3DSPARSE_LIB", os.path.join(PKG_ROOT, "lib", "libmi3dsparse.so"))

P, I, I64, F, D, SZ = c_void_p, c_int, c_int64, c_float, c_double, c_size_t


class WeightImage(ctypes.Structure):
    """msp_weight_image (include/mi3dsparse.h)."""
    _fields_ = [("wt", c_void_p), ("img", c_void_p), ("units", c_int64), ("bytes", c_int64), ("kind", ctypes.c_int32),
                ("K", ctypes.c_int32), ("c_in", ctypes.c_int32), ("c_out", ctypes.c_int32), ("p", ctypes.c_int32),
                ("wlay", ctypes.c_int32)]

class BnEpilogue(ctypes.Structure):
    """msp_bn_epilogue (include/mi3dsparse.h)."""
    _fields_ = [("partial", c_void_p), ("x", c_void_p), ("stats", c_void_p), ("leak", c_float)]


# name -> (restype, argtypes); mirrors include/mi3dsparse.h one to one
PROTOTYPES = {
    "msp_abi_version": (I, []),
    "msp_last_error": (ctypes.c_char_p, []),
    "msp_point_keys": (I, [P, I64, I64, I, I64, P, P, P, P]),
    "msp_batch_starts": (I, [P, I64, I64, I64, P, P]),
    "msp_sort_workspace_size": (SZ, [I64, I]),
    "msp_sort_pairs": (I, [P, P, P, P, I64, I, P, SZ, P]),
    "msp_scan_workspace_size": (SZ, [I64]),
    "msp_segment": (I, [P, I64, I, P, P, P, P, P, P, P, SZ, P]),
    "msp_hash_capacity": (I64, [I64]),
    "msp_hash_build": (I, [P, I64, P, I64, P]),
    "msp_subm_map": (I, [P, I64, I, I64, I, P, I64, P, P]),
    "msp_subm_map_workspace_size": (SZ, [I64, I]),
    "msp_subm_map_counted": (I, [P, I64, I, I64, I, P, I64, P, P, P, SZ, P]),
    "msp_down_map": (I, [P, I64, P, I, I, P, I64, P]),
    "msp_pair_lists": (I, [P, I, I64, P, P, I64, P, P, SZ, P]),
    "msp_tile_rulebook": (I, [P, I, I64, I, P, P, P, P, I64, P, SZ, P]),
    "msp_decode_keys": (I, [P, I64, I, P, P]),
    "msp_tile_local_workspace_size": (SZ, [I64, I]),
    "msp_tile_local": (I, [P, I, I64, I, P, P, I64, P, P, P, P, SZ, P]),
    "msp_conv_local_preferred": (I, [I64, I, I]),
    "msp_wgrad_chunk_ok": (I, [I64, I, I, I]),
    "msp_wgrad_chunk_preferred": (I, [I64, I, I, I]),
    "msp_wgrad_chunk_ranges": (I64, [I64, I, I]),
    "msp_wgrad_chunk_cap": (I64, []),
    "msp_wgrad_chunk_index": (I, [P, P, P, I64, P, P, P, P, P]),
    "msp_local_chunk_index": (I, [P, P, I, I64, P, P, P, I64, P, SZ, P]),
    "msp_conv_wgrad_chunk": (I, [P, I, P, I, I, I, P, P, P, P, P, I64, I64, P, P, P]),
    "msp_wgrad_far_workspace_size": (SZ, [I64]),
    "msp_wgrad_far_list": (I, [P, P, P, I64, I64, P, P, P, SZ, P]),
    "msp_conv_wgrad_far": (I, [P, I, P, I, I, P, P, P, P, I64, P, P]),
    "msp_conv_local_workspace_size": (SZ, [I, I, I]),
    "msp_conv_local": (I, [P, I, P, I, I, I, I, P, P, P, P, P, I64, P, P, SZ, P]),
    "msp_conv_tile_rows": (I, [I64, I, I]),
    "msp_conv_tile_form": (I, [I64, I, I, I]),
    "msp_conv_tile_workspace_size": (SZ, [I64, I, I, I, I]),
    "msp_conv_tile": (I, [P, I, P, I, I, I, I, P, P, P, P, I64, P, P, SZ, P]),
    "msp_conv_nbr_preferred": (I, [I64, I, I]),
    "msp_conv_nbr_workspace_size": (SZ, [I, I, I]),
    "msp_conv_nbr": (I, [P, I, P, I, I, I, P, P, I64, P, P, SZ, P]),
    "msp_dense_order_workspace_size": (SZ, [I64, I, I]),
    "msp_dense_order": (I, [P, I, I64, I, P, P, P, SZ, P]),
    "msp_conv_pairs": (I, [P, I, P, I, I, P, P, P, P, I64, P, P]),
    "msp_wgrad_pieces": (I64, [I64, I, I, I]),
    "msp_conv_wgrad": (I, [P, I, P, I, P, P, P, I, I64, P, P, P]),
    "msp_conv_weight_image": (I, [I, I64, I, I, I, I, P]),
    "msp_split_weight_images": (I, [P, I, P, I64, P]),
    "msp_conv_narrow_in_ok": (I, [I, I, I]),
    "msp_conv_narrow_in": (I, [P, I, P, I, I, P, I64, P, P]),
    "msp_conv_wgrad_narrow_parts": (I64, [I64, I, I, I]),
    "msp_conv_wgrad_narrow_in": (I, [P, I, P, I, P, I, I64, I64, P, P, P]),
    "msp_bn_partials": (I64, [I64, I]),
    "msp_bn_stats": (I, [P, I64, I, P, P]),
    "msp_bn_finalize": (I, [P, I64, I, D, D, I, P, P, P, P, P, P]),
    "msp_bn_apply": (I, [P, I64, I, P, F, P, P]),
    "msp_bn_bwd_stats": (I, [P, P, I64, I, P, F, P, P]),
    "msp_bn_bwd_apply": (I, [P, P, I64, I, P, P, P, F, I, P, P, P, P]),
    "msp_bn_bwd_apply_add": (I, [P, P, I64, I, P, P, P, F, I, P, P, P, P, P]),
    "msp_bn_bwd_apply_split": (I, [P, P, I64, I, P, P, P, F, I, P, I, P, P, P, P, P]),
    "msp_conv_pairs_x6_workspace_size": (SZ, [I, I, I]),
    "msp_conv_pairs_x6": (I, [P, I, P, I, I, P, P, P, P, I64, P, P, SZ, P]),
    "msp_adam_chunks": (I64, [I64]),
    "msp_adam_step": (I, [P, P, P, I, I64, P, I, D, D, D, D, D, P]),
    "msp_add_bn_stats": (I, [P, P, I64, I, P, P, P]),
    "msp_conv_bn_parts": (I64, [I64]),
    "msp_conv_local_bn": (I, [P, I, P, I, I, I, I, P, P, P, P, P, I64, P, P, SZ, P, P]),
    "msp_conv_tile_bn": (I, [P, I, P, I, I, I, I, P, P, P, P, I64, P, P, SZ, P, P]),
    "msp_bn_finalize_cm": (I, [P, I64, I64, I, D, D, I, P, P, P, P, P, P]),
    "msp_bn_bwd_apply_cm": (I, [P, P, I64, I, P, I64, P, P, F, I, P, P, P, P, P]),
    "msp_join_cols": (I, [P, I, P, I, I64, P, P, P]),
    "msp_split_cols": (I, [P, I64, I, I, P, P, P]),
    "msp_nin_gemm_ok": (I, [I64, I, I]),
    "msp_nin_gemm_form": (I, [I64, I, I]),
    "msp_nin_gemm_workspace_size": (SZ, [I, I]),
    "msp_nin_gemm": (I, [P, I64, I, P, I, P, P, SZ, P]),
    "msp_input_avg_fwd": (I, [P, I, P, P, I64, P, P]),
    "msp_input_avg_bwd": (I, [P, I, P, P, I64, P, P]),
    "msp_output_fwd": (I, [P, I, P, I64, P, P]),
    "msp_output_bwd": (I, [P, I, P, P, I64, P, P]),
    "msp_unpool_fwd": (I, [P, I, P, I64, P, P]),
    "msp_unpool_bwd": (I, [P, I, P, I64, P, P]),
    "msp_maxpool_fwd": (I, [P, I, P, I64, P, P, P]),
    "msp_maxpool_bwd": (I, [P, I, P, I64, P, P]),
    "msp_scene_mean_workspace_size": (SZ, [I64, I, I]),
    "msp_scene_mean_fwd": (I, [P, I, P, I64, I, P, I, P, P, P, P, SZ, P]),
    "msp_scene_mean_bwd": (I, [P, I, P, I64, I, P, P, P, P]),
    "msp_point_rows_bias": (I, [P, I64, I, P, P, I64, P, P]),
    "msp_index_add_workspace_size": (SZ, [I64, I64]),
    "msp_index_add_rows": (I, [P, I64, I, P, P, I64, P, SZ, P]),
    "msp_merge_workspace_size": (SZ, [I, I64]),
    "msp_merge": (I, [P, P, P, P, I, I64, I, D, P, P, P, P, P, P, I, P, P, P, P, I64, P, P, P, SZ, P]),
}

_lib = None


def load():
    """Load the library once; raise if it is absent (no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.isfile(LIB_PATH):
            raise RuntimeError(
                f"mi3dsparse: {LIB_PATH} not found - build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                " (there is no CPU fallback)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("mi3dsparse kernels need HIP device tensors (got a CPU tensor); there is no CPU path")
    return t.data_ptr()


# the current stream's raw handle without a torch.cuda.Stream object per call (a step asks ~170 times; the Stream
# wrapper cost ~5 us each, measurable on the host-bound configurations).  MI3DSPARSE_TORCH_STREAM=1: the public path.
_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None) \
    if os.environ.get("MI3DSPARSE_TORCH_STREAM") != "1" else None


def stream(device=None):
    if _RAW_STREAM is not None:
        if isinstance(device, torch.device) and device.index is not None:
            return _RAW_STREAM(device.index)
        if isinstance(device, int):
            return _RAW_STREAM(device)
        return _RAW_STREAM(torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


_SYNC = os.environ.get("MI3DSPARSE_SYNC") == "1"  # debugging: synchronise after every call


def call(name, *args):
    """Invoke an int-returning entry point; raise RuntimeError on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.msp_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")
    if _SYNC:
        try:
            torch.cuda.synchronize()
        except Exception as e:  # name the entry point whose kernels faulted
            raise RuntimeError(f"{name}: device fault after this call: {e}") from e


_QUERIES = {}


def query(name, *args):
    """Invoke a size/capacity query that returns a value.  The queries are pure functions of their arguments
    (the device's CU count aside), so results are memoised: a training step asks the same few hundred
    questions every step, at a ctypes round trip each."""
    key = (name,) + tuple(a.value if isinstance(a, ctypes._SimpleCData) else a for a in args)
    r = _QUERIES.get(key)
    if r is None:
        if len(_QUERIES) > 1 << 16:
            _QUERIES.clear()
        r = _QUERIES[key] = getattr(load(), name)(*args)
    return r


# --------------------------------------------------------------- GPU event hooks
# bench.py installs a recorder here to time the dominant kernel live (HIP
# events on the launch stream) and to sum its algorithmic FLOPs.
_recorder = None


def set_recorder(rec):
    global _recorder
    _recorder = rec


def recorder():
    return _recorder
