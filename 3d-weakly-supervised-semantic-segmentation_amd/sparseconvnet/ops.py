"""autograd Functions over libmi3dsparse.

Each Function owns the saved tensors of its backward (features, weights,
rulebooks); every forward and backward pass is one or more C-ABI calls on the
current HIP stream.  Channel counts that are not multiples of 16 (the 3-channel
colour input of the first SubmanifoldConvolution, models/SparseConvNet.py:62)
are zero-padded to the MFMA chunk width here and sliced back.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn.functional as F

from . import _lib
from . import weight_images as _wimg
from ._lib import call, ptr

_EMPTY = {}
# diagnosis (bench.py per-kind breakdowns): recorded kinds carry the call's shape, "[c_in x c_out : rows]"
_SHAPES = os.environ.get("MI3DSPARSE_KIND_SHAPES") == "1"


def _shape(kind, c_in, c_out, n):
    return f"{kind}[{c_in}x{c_out}:{n}]" if _SHAPES else kind


def _stream(t):
    return _lib.stream(t.device)


def _pad16(c):
    return (c + 15) // 16 * 16


def _pad_cols(x, c):
    return x if x.size(1) == c else F.pad(x, (0, c - x.size(1)))


def _check_feats(x):
    if not x.is_cuda:
        raise RuntimeError("sparseconvnet (mi3dsparse): features must be on a HIP device; there is no CPU path")
    if x.dtype != torch.float32:
        raise TypeError(f"sparseconvnet (mi3dsparse): features must be float32, got {x.dtype}")


def _pad_weight(w, cin_p, cout_p):
    K, cin, cout = w.shape
    if cin == cin_p and cout == cout_p:
        return w.contiguous()
    return F.pad(w, (0, cout_p - cout, 0, cin_p - cin))


def _workspace(entry, wt, n_rows, K, c_in, c_out, flip, wsb, device):
    """(workspace tensor, its bytes, flip) for a convolution call: the step's prepared weight image when
    sparseconvnet.weight_images is on and holds a fresh one (flip bit 2: the split is skipped), else a new
    workspace the call splits its weights into."""
    wi = _wimg.active()
    if wi is not None:
        img = wi.lookup(entry, wt, n_rows, K, c_in, c_out, flip)
        if img is not None:
            return img, img.numel(), flip | 4
    return torch.empty(max(wsb // 4, 1), dtype=torch.float32, device=device), wsb, flip


def _record(kind, flops, fn, nbytes=0):
    """Run fn(); when bench.py installed a recorder, bracket it with HIP
    events on the current stream and account its algorithmic FLOPs and
    compulsory bytes."""
    rec = _lib.recorder()
    if rec is None:
        return fn()
    return rec.run(kind, flops, fn, nbytes)


# ------------------------------------------------------------------ convolution helpers
def conv_form(rules, n_rows, c_in, c_out, K):
    """Which form (and so which rulebook) the convolution over `rules` takes for these sizes: "local", "nbr", or
    the tile height of msp_conv_tile -- the library's preference queries."""
    nbr = getattr(rules, "nbr", None)  # submanifold rules carry the neighbour map
    if nbr is not None and n_rows and K <= 27 and \
            int(_lib.query("msp_conv_local_preferred", _lib.I64(n_rows), c_in, c_out)):
        return "local"
    if nbr is not None and n_rows and int(_lib.query("msp_conv_nbr_preferred", _lib.I64(n_rows), c_in, c_out)):
        return "nbr"
    return int(_lib.query("msp_conv_tile_rows", _lib.I64(n_rows), c_in, c_out))


def prepare(rules, purpose, c_in, c_out):
    """Build the rulebooks a convolution ("conv": forward / backward-data) or a submanifold weight gradient
    ("wgrad") over `rules` will use for these channel counts, for the rules' own row count (Metadata.replay:
    a prefetched batch gets exactly what its sizes select, even when they cross a threshold the previous
    batch's did not)."""
    n, K = rules._n, rules.K
    if purpose == "conv":
        f = conv_form(rules, n, c_in, c_out, K)
        if f == "local":
            rules.local()
        elif f == "nbr":
            rules.dense_order()
        else:
            rules.tiles_for(f)
    elif purpose == "wgrad":
        if int(_lib.query("msp_wgrad_chunk_preferred", _lib.I64(n), K, c_in, c_out)):
            if rules.wgrad_index() is not None:
                return
        rules.pairs.fill()
    elif purpose == "pairs":  # strided convolution backward, deconvolution: one contribution per pair
        rules.pairs.fill()


# ------------------------------------------------------------------ BatchNorm statistics in convolution epilogues
# The BN -> SubM -> BN -> SubM chains of the residual blocks (models/SparseConvNet.py:63-69): the submanifold
# convolution that feeds a training-mode BatchNorm leaves that BN's forward sums in its epilogue, and the
# backward-data of the convolution a BatchNorm feeds leaves that BN's backward sums (msp_bn_epilogue), so the BN
# skips its own statistics pass over the rows.  Off by default (MI3DSPARSE_BN_EPILOGUE=1 turns it
# on): the BN family drops from 9.0 to 7.5 ms/step but the convolutions' epilogues cost more than that -- 50.08-50.20
# vs 49.80-49.89 ms/step, interleaved on one box (profiles/r06/ab_r06g_bnepi_on_off.txt).
FUSE_BN_STATS = os.environ.get("MI3DSPARSE_BN_EPILOGUE", "0") == "1"


class BnParts:
    """Channel-major BatchNorm partial sums [2][C][P] (+ the [2][C] tail msp_bn_bwd_apply_cm writes) that a
    convolution epilogue fills, one slot per 128-row tile; `written` once a call filled them."""
    __slots__ = ("buf", "P", "C", "written")

    def __init__(self, C, n_rows, device):
        self.C = int(C)
        self.P = int(_lib.query("msp_conv_bn_parts", _lib.I64(n_rows)))
        self.buf = torch.empty(max(2 * self.C * (self.P + 1), 1), dtype=torch.float64, device=device)
        self.written = False


class BnLink:
    """A training-mode BatchNorm-ReLU whose output a submanifold convolution consumes: the BN's forward fills
    x / stats; the convolution's backward-data, when its form has the epilogue, leaves the BN's backward sums in
    `bwd` = (the gradient tensor it returned, BnParts); the BN's backward uses them when the gradient it receives
    is that very tensor (one consumer)."""
    __slots__ = ("leak", "x", "stats", "bwd")

    def __init__(self, leak):
        self.leak = float(leak)
        self.x = self.stats = self.bwd = None


def bn_epi_ok(rules, n_rows, c_in, c_out, K):
    """Whether the convolution over `rules` for these sizes runs a form with the BatchNorm epilogue (the
    tile-local form, or the per-wave tiles of msp_conv_tile)."""
    if not n_rows:
        return False
    f = conv_form(rules, n_rows, c_in, c_out, K)
    if f == "local":
        return True
    if f == "nbr":
        return False
    return int(_lib.query("msp_conv_tile_form", _lib.I64(n_rows), c_in, c_out, f)) == 1


def _epi_arg(epi):
    """ctypes pointer to an msp_bn_epilogue for epi = (BnParts, BN input x or None, BN stats or None, leak)."""
    parts, xb, stats, leak = epi
    e = _lib.BnEpilogue(parts.buf.data_ptr(), xb.data_ptr() if xb is not None else None,
                        stats.data_ptr() if stats is not None else None, float(leak))
    return ctypes.byref(e)  # keeps e alive with the pointer


def conv_tile(x, wt, K, flip, c_out, rules, n_rows, kind="conv_tile", flops=0, epi=None):
    """Output-stationary convolution over the rulebook's tile form; the tile
    height (and so which rulebook) is the library's choice for these channel
    counts (msp_conv_tile_rows).  epi: the BatchNorm epilogue (bn_epi_ok must hold)."""
    c_in = x.size(1)
    rules.note_use("conv", c_in, c_out)
    f = conv_form(rules, n_rows, c_in, c_out, K)
    if f == "local":
        return conv_local(x, wt, K, flip, c_out, rules, n_rows, kind, flops, epi)
    if epi is not None and (f == "nbr" or not n_rows or
                            int(_lib.query("msp_conv_tile_form", _lib.I64(n_rows), c_in, c_out, f)) != 1):
        raise RuntimeError("conv_tile: the BatchNorm epilogue needs the tile-local or per-wave form (bn_epi_ok)")
    if f == "nbr":
        perm, nbr_p = rules.dense_order()
        return conv_nbr(x, wt, K, flip, c_out, nbr_p, n_rows, kind, flops, perm)
    tr = f
    tiles = rules.tiles_for(tr)
    out = torch.empty((max(n_rows, 1), c_out), dtype=torch.float32, device=x.device)
    if n_rows:
        # the contraction msp_conv_tile runs on 128-row tiles: bf16 MFMA over
        # exact three-piece operand splits (per-wave tiles for narrow outputs)
        form = int(_lib.query("msp_conv_tile_form", _lib.I64(n_rows), c_in, c_out, tr))
        kind = _shape(kind + {1: "/x6r", 2: "/x6d"}.get(form, "/f32"), c_in, c_out, n_rows)
        wsb = int(_lib.query("msp_conv_tile_workspace_size", _lib.I64(n_rows), K, c_in, c_out, tr))
        ws, wsb, flip = _workspace(0, wt, n_rows, K, c_in, c_out, int(flip), wsb, x.device)
        # compulsory bytes: input rows, output rows, weights, rulebook (chunk
        # offsets, 16 x (int32 src + uint16 row) per chunk, tile starts)
        nbytes = 4 * (x.size(0) * c_in + n_rows * c_out + K * c_in * c_out) + \
            tiles["n_chunks"] * (1 + 16 * 6) + 8 * (tiles["tile_start"].numel())
        if epi is None:
            _record(kind, flops, lambda: call(
                "msp_conv_tile", ptr(x), c_in, ptr(wt), K, int(flip), c_out, tr, ptr(tiles["tile_start"]),
                ptr(tiles["chunk_off"]), ptr(tiles["chunk_src"]), ptr(tiles["chunk_row"]), n_rows, ptr(out),
                ptr(ws), wsb, _stream(x)), nbytes)
        else:  # + the epilogue's read of the BN input rows (backward)
            ea = _epi_arg(epi)
            _record(kind, flops, lambda: call(
                "msp_conv_tile_bn", ptr(x), c_in, ptr(wt), K, int(flip), c_out, tr, ptr(tiles["tile_start"]),
                ptr(tiles["chunk_off"]), ptr(tiles["chunk_src"]), ptr(tiles["chunk_row"]), n_rows, ptr(out),
                ptr(ws), wsb, ea, _stream(x)), nbytes + (4 * n_rows * c_out if epi[1] is not None else 0))
            epi[0].written = True
    return out[:n_rows]


def conv_local(x, wt, K, flip, c_out, rules, n_rows, kind="conv_local", flops=0, epi=None):
    """Submanifold convolution over the tile-local rulebook (SubmRules.local): each 128-row tile's distinct
    input rows staged in LDS and split once (msp_conv_local); epi: the BatchNorm epilogue (msp_conv_local_bn)."""
    c_in = x.size(1)
    loc = rules.local()
    out = torch.empty((max(n_rows, 1), c_out), dtype=torch.float32, device=x.device)
    wsb = int(_lib.query("msp_conv_local_workspace_size", K, c_in, c_out))
    ws, wsb, flip = _workspace(1, wt, n_rows, K, c_in, c_out, int(flip), wsb, x.device)
    # compulsory bytes: input rows, output rows, weights, the tile-local rulebook
    nbytes = 4 * (x.size(0) * c_in + n_rows * c_out + K * c_in * c_out) + \
        4 * loc["total"] + 2 * K * loc["n_tiles"] * loc["tile_rows"] + 4 * loc["n_tiles"] * loc["tile_rows"]
    if epi is None:
        _record(_shape(kind + "/x6s", c_in, c_out, n_rows), flops, lambda: call(
            "msp_conv_local", ptr(x), c_in, ptr(wt), K, int(flip), c_out, loc["tile_rows"], ptr(loc["lidx"]),
            ptr(loc["u_start"]), ptr(loc["u_rows"]), ptr(loc["perm"]), ptr(loc.get("wave_off")), n_rows, ptr(out),
            ptr(ws), wsb, _stream(x)),
            nbytes)
    elif n_rows:  # + the epilogue's read of the BN input rows (backward)
        ea = _epi_arg(epi)
        _record(_shape(kind + "/x6s", c_in, c_out, n_rows), flops, lambda: call(
            "msp_conv_local_bn", ptr(x), c_in, ptr(wt), K, int(flip), c_out, loc["tile_rows"], ptr(loc["lidx"]),
            ptr(loc["u_start"]), ptr(loc["u_rows"]), ptr(loc["perm"]), ptr(loc.get("wave_off")), n_rows, ptr(out),
            ptr(ws), wsb, ea, _stream(x)),
            nbytes + (4 * n_rows * c_out if epi[1] is not None else 0))
        epi[0].written = True
    return out[:n_rows]


# One contribution per output row (deconvolution forward, strided backward-data) on the split-bf16 MFMAs
# (msp_conv_pairs_x6, round 6) instead of the exact fp32 16x16x4 MFMA chains of msp_conv_pairs.
PAIRS_X6 = os.environ.get("MI3DSPARSE_PAIRS_X6", "1") == "1"
PAIRS_FORM = "x6" if PAIRS_X6 else "f32"


def conv_pairs(x, wt, K, c_out, pairs, pin, pout, n_out, kind="pairs", flops=0):
    """out[pout[p]] = wt[o]^T x[pin[p]] (wt [K][c_out][c_in]), one pair per output row."""
    out = torch.empty((max(n_out, 1), c_out), dtype=torch.float32, device=x.device)
    if pairs.n_chunks:
        c_in = x.size(1)
        # compulsory bytes: source rows, output rows, weights, the pair lists
        nbytes = 4 * (x.size(0) * c_in + n_out * c_out + K * c_in * c_out) + 8 * pairs.total
        if PAIRS_X6 and c_in % 16 == 0 and c_out % 16 == 0:
            wsb = int(_lib.query("msp_conv_pairs_x6_workspace_size", K, c_in, c_out))
            ws = torch.empty(max(wsb, 16) // 4 + 4, dtype=torch.float32, device=x.device)
            _record(kind + "/x6", flops, lambda: call(
                "msp_conv_pairs_x6", ptr(x), c_in, ptr(wt), K, c_out, ptr(pin), ptr(pout), ptr(pairs.off_start),
                ptr(pairs.chunk_start), pairs.n_chunks, ptr(out), ptr(ws), wsb, _stream(x)), nbytes)
        else:
            _record(kind + "/f32", flops, lambda: call(
                "msp_conv_pairs", ptr(x), c_in, ptr(wt), K, c_out, ptr(pin), ptr(pout), ptr(pairs.off_start),
                ptr(pairs.chunk_start), pairs.n_chunks, ptr(out), _stream(x)), nbytes)
    return out[:n_out]


# Strided-convolution and deconvolution weight gradients on the chunk form over the child map (round 6, opt-in:
# MI3DSPARSE_STRIDED_WGRAD_CHUNK=1).  Measured slower than the per-offset pair lists on the headline step: the kernels
# 2.18 / 2.30 vs 1.94 / 2.01 ms per 5 steps (a 128-coarse-row tile names ~2.4 x 128 fine rows, often past the 448
# staged, and 8 offsets leave the k-steps short), and the child maps' tile rulebooks, distinct-row lists and far-rule
# lists add ~9 ms of prefetch host time and side-stream work: 61.0 vs 50.0-50.1 ms/step
# (profiles/r06/ab_r06k_strided_wgrad_chunk.txt).  Kept for its tests (the far-rule path on dense children).
STRIDED_WGRAD_CHUNK = os.environ.get("MI3DSPARSE_STRIDED_WGRAD_CHUNK", "0") == "1"

_WGRAD_SIDE = {}
# True: every weight gradient on a side stream beside the backward-data (bench.py --concurrent-wgrad).
# Off by default: it saved 0.3 ms of 66.9 per step (round 2, eager), inside the box-to-box spread, and the
# co-running kernels stretch each other's event-timed durations (the conv roofline reads low).
WGRAD_CONCURRENT = False
# Levels below this many rows run their weight gradient beside the backward-data (bench.py --wgrad-side-rows).
# Off: although neither fills the chip below ~10^4 rows, the graph-captured step measured 54.6-54.8 ms with it
# at 2^14 rows and 54.6 at 2^16, against 54.2 without (profiles/r03/args_r03_wgrad_side.log).
WGRAD_SIDE_ROWS = 0


def _on_side(x, rows, fn):
    """fn() on a side stream ordered after the work already queued on the current stream, so it runs
    concurrently with what is launched next on the current stream, when WGRAD_CONCURRENT or the level has
    fewer than WGRAD_SIDE_ROWS rows; else on the current stream.  Returns (result, join): join() makes the
    current stream wait for it -- call it before the backward returns, so everything after this autograd node
    is ordered after it as well."""
    if not (WGRAD_CONCURRENT or rows < WGRAD_SIDE_ROWS) or not x.is_cuda:
        return fn(), lambda: None
    dev = x.device
    cur = torch.cuda.current_stream(dev)
    side = _WGRAD_SIDE.get(dev.index)
    if side is None:
        side = _WGRAD_SIDE[dev.index] = torch.cuda.Stream(dev)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        out = fn()
        ev = torch.cuda.Event()
        ev.record(side)

    def join():
        cur.wait_event(ev)
        if out is not None:
            out.record_stream(cur)
    return out, join


def conv_wgrad_async(x, dy, pairs, pin, pout, K, flops=None, kind="wgrad"):
    """conv_wgrad beside the backward-data launched next on the current stream (_on_side: both are
    latency-bound gathers at 2-3 waves per SIMD; co-running fills the chip).  Returns (dw, join)."""
    return _on_side(x, dy.size(0), lambda: conv_wgrad(x, dy, pairs, pin, pout, K, kind, flops=flops))


def conv_wgrad(x, dy, pairs, pin, pout, K, kind="wgrad", flops=None):
    c_in, c_out = x.size(1), dy.size(1)
    dw = torch.empty((K, c_in, c_out), dtype=torch.float32, device=x.device)
    n_pieces = int(_lib.query("msp_wgrad_pieces", _lib.I64(pairs.total), K, c_in, c_out))
    slab = torch.empty((n_pieces, K, c_in, c_out), dtype=torch.float32, device=x.device)
    if flops is None:
        flops = 2.0 * pairs.total * c_in * c_out
    # compulsory bytes: x and dy rows, the pair lists, dW
    nbytes = 4 * (x.size(0) * c_in + dy.size(0) * c_out + K * c_in * c_out) + 8 * pairs.total
    _record(_shape(kind + "/x6", c_in, c_out, dy.size(0)), flops, lambda: call(
        "msp_conv_wgrad", ptr(x), c_in, ptr(dy), c_out, ptr(pin), ptr(pout), ptr(pairs.off_start), K,
        n_pieces, ptr(slab), ptr(dw), _stream(x)), nbytes)
    return dw


def conv_wgrad_chunk(x, dy, rules, K, kind="wgrad", flops=None):
    """Submanifold weight gradient over the 128-row tile rulebook (SubmRules.wgrad_index): per tile the distinct
    x rows and the 128 dy rows staged in LDS once per 32 x 32 channel slice, the compacted chunks as MFMA
    k-steps (msp_conv_wgrad_chunk); partial sums per tile range added in order; then the rules of rows past a
    tile's staged capacity, if any (msp_conv_wgrad_far)."""
    idx = rules.wgrad_index(wait=True)
    c_in, c_out = x.size(1), dy.size(1)
    n = dy.size(0)
    tiles = idx["tiles"]
    ranges = int(_lib.query("msp_wgrad_chunk_ranges", _lib.I64(n), c_in, c_out))
    dw = torch.empty((K, c_in, c_out), dtype=torch.float32, device=x.device)
    slab = torch.empty((ranges, K, c_in, c_out), dtype=torch.float32, device=x.device)
    if flops is None:
        flops = 2.0 * rules.n_rules * c_in * c_out
    # compulsory bytes: x and dy rows, the rulebook (one packed word per chunk entry, chunk offsets, tile
    # starts), the tiles' distinct-row lists, dW
    nbytes = 4 * (x.size(0) * c_in + n * c_out + K * c_in * c_out) + \
        tiles["n_chunks"] * (1 + 16 * 4) + 8 * tiles["tile_start"].numel() + 4 * idx["u_rows"].numel()
    _record(_shape(kind + "/x6c", c_in, c_out, n), flops, lambda: call(
        "msp_conv_wgrad_chunk", ptr(x), c_in, ptr(dy), c_out, K, tiles["tile_rows"], ptr(tiles["tile_start"]),
        ptr(tiles["chunk_off"]), ptr(idx["chunk_lr"]), ptr(idx["u_start"]), ptr(idx["u_rows"]), n, ranges,
        ptr(slab), ptr(dw), _stream(x)), nbytes)
    if idx["n_far"]:
        call("msp_conv_wgrad_far", ptr(x), c_in, ptr(dy), c_out, K, ptr(tiles["chunk_src"]), ptr(tiles["chunk_row"]),
             ptr(idx["far_key"]), ptr(idx["far_tile"]), idx["n_far"], ptr(dw), _stream(x))
    return dw


def conv_nbr(x, wt, K, flip, c_out, nbr, n_rows, kind="conv_nbr", flops=0, perm=None):
    """Dense row-group form of the submanifold convolution straight from the
    neighbour map nbr[K][n_rows] (msp_conv_nbr: no tile rulebook); with perm,
    nbr is the map permuted by it (SubmRules.dense_order)."""
    c_in = x.size(1)
    out = torch.empty((max(n_rows, 1), c_out), dtype=torch.float32, device=x.device)
    wsb = int(_lib.query("msp_conv_nbr_workspace_size", K, c_in, c_out))
    ws, wsb, flip = _workspace(2, wt, n_rows, K, c_in, c_out, int(flip), wsb, x.device)
    # compulsory bytes: input rows, output rows, weights, the neighbour map (+ row order)
    nbytes = 4 * (x.size(0) * c_in + n_rows * c_out + K * c_in * c_out + K * n_rows + (n_rows if perm is not None else 0))
    _record(kind + "/x6g", flops, lambda: call(
        "msp_conv_nbr", ptr(x), c_in, ptr(wt), K, int(flip), c_out, ptr(nbr), ptr(perm) if perm is not None else None,
        n_rows, ptr(out), ptr(ws), wsb, _stream(x)), nbytes)
    return out[:n_rows]


# ------------------------------------------------------------------ submanifold
class SubmanifoldConvFunction(torch.autograd.Function):
    """out[i] = sum_o W[o]^T x[nbr(i, o)] over the active set."""

    @staticmethod
    def forward(ctx, x, weight, rules, link=None, parts=None):
        """link: BnLink of the BatchNorm whose output x is (its backward sums from this convolution's
        backward-data); parts: BnParts for the forward sums of the output, for the BatchNorm it feeds (filled
        when the form has the epilogue: parts.written)."""
        _check_feats(x)
        K, _, cin, cout = weight.shape
        V = x.size(0)
        ctx.link = None
        nbr = getattr(rules, "nbr", None)
        if nbr is not None and int(_lib.query("msp_conv_narrow_in_ok", K, cin, cout)):
            # the colour input layer (c_in <= 4): straight from the neighbour map, no channel padding
            xc, wc = x.contiguous(), weight.reshape(K, cin, cout).contiguous()
            out = torch.empty((max(V, 1), cout), dtype=torch.float32, device=x.device)
            if V:
                nbytes = 4 * (V * cin + V * cout + K * cin * cout + K * V)
                _record(_shape("subm_fwd/f32n", cin, cout, V), 2.0 * rules.n_rules * cin * cout, lambda: call(
                    "msp_conv_narrow_in", ptr(xc), cin, ptr(wc), K, cout, ptr(nbr), V, ptr(out), _stream(x)), nbytes)
            ctx.save_for_backward(xc, wc)
            ctx.rules, ctx.dims, ctx.narrow = rules, (cin, cout), True
            return out[:V]
        cin_p, cout_p = _pad16(cin), _pad16(cout)
        xp = _pad_cols(x.contiguous(), cin_p)
        wp = _pad_weight(weight.reshape(K, cin, cout), cin_p, cout_p)
        # flip bit 1: the weights in their own [K][c_in][c_out] layout (no transposed copy)
        epi = None
        if parts is not None and cout_p == cout and parts.C == cout and bn_epi_ok(rules, V, cin_p, cout_p, K):
            epi = (parts, None, None, 0.0)
        out = conv_tile(xp, wp, K, 2, cout_p, rules, V, "subm_fwd",
                        2.0 * rules.n_rules * cin * cout, epi=epi)
        ctx.save_for_backward(xp, wp)
        ctx.rules, ctx.dims, ctx.narrow = rules, (cin, cout), False
        if link is not None and cin_p == cin:
            ctx.link = link
        return out if cout_p == cout else out[:, :cout].contiguous()

    @staticmethod
    def backward(ctx, gout):
        if ctx.narrow:
            return SubmanifoldConvFunction._backward_narrow(ctx, gout)
        xp, wp = ctx.saved_tensors
        rules, (cin, cout) = ctx.rules, ctx.dims
        K, cin_p, cout_p = wp.shape
        g = _pad_cols(gout.contiguous(), cout_p)
        dx = dw = None
        join = None
        if ctx.needs_input_grad[1]:
            V = xp.size(0)
            dwp = None
            rules.note_use("wgrad", cin_p, cout_p)
            flops = 2.0 * rules.n_rules * cin * cout
            if int(_lib.query("msp_wgrad_chunk_preferred", _lib.I64(V), K, cin_p, cout_p)) and \
                    rules.wgrad_index(wait=True) is not None:
                dwp, join = _on_side(xp, V, lambda: conv_wgrad_chunk(xp, g, rules, K, flops=flops))
            if dwp is None:  # pair lists (beside the backward-data on small levels or when WGRAD_CONCURRENT)
                p = rules.pairs  # (built by the prefetch when this batch's sizes select them: ops.prepare)
                dwp, join = conv_wgrad_async(xp, g, p, p.pair_in, p.pair_out, K, flops)
            dw = dwp[:, :cin, :cout].reshape(K, 1, cin, cout)
        if ctx.needs_input_grad[0]:
            V = xp.size(0)
            link, epi = ctx.link, None
            if link is not None and link.x is not None and bn_epi_ok(rules, V, cout_p, cin_p, K):
                # the BatchNorm that produced x gets its backward sums from this call's epilogue
                epi = (BnParts(cin_p, V, g.device), link.x, link.stats, link.leak)
            dxp = conv_tile(g, wp, K, 1, cin_p, rules, V, "subm_bwd_data",
                            2.0 * rules.n_rules * cin * cout, epi=epi)
            if epi is not None:
                link.bwd = (dxp, epi[0])
            dx = dxp if cin_p == cin else dxp[:, :cin]
        if join is not None:
            join()
        ctx.link = None
        return dx, dw, None, None, None

    @staticmethod
    def _backward_narrow(ctx, gout):
        x, w = ctx.saved_tensors
        rules, (cin, cout) = ctx.rules, ctx.dims
        K, V = w.size(0), x.size(0)
        g = gout.contiguous()
        dx = dw = None
        if ctx.needs_input_grad[1]:
            parts = int(_lib.query("msp_conv_wgrad_narrow_parts", _lib.I64(V), K, cin, cout))
            slab = torch.empty((parts, K, cin, cout), dtype=torch.float32, device=x.device)
            dw = torch.empty((K, cin, cout), dtype=torch.float32, device=x.device)
            nbytes = 4 * (V * cin + V * cout + K * cin * cout + K * V)
            _record(_shape("wgrad/f32n", cin, cout, V), 2.0 * rules.n_rules * cin * cout, lambda: call(
                "msp_conv_wgrad_narrow_in", ptr(x), cin, ptr(g), cout, ptr(rules.nbr), K, V, parts, ptr(slab),
                ptr(dw), _stream(x)), nbytes)
            dw = dw.reshape(K, 1, cin, cout)
        if ctx.needs_input_grad[0]:  # (the input layer's features rarely need a gradient): padded tile path
            cin_p, cout_p = _pad16(cin), _pad16(cout)
            wp = _pad_weight(w, cin_p, cout_p)
            dxp = conv_tile(_pad_cols(g, cout_p), wp, K, 1, cin_p, rules, V, "subm_bwd_data",
                            2.0 * rules.n_rules * cin * cout)
            dx = dxp[:, :cin]
        return dx, dw, None, None, None


# ------------------------------------------------------------------ strided convolution
class ConvolutionFunction(torch.autograd.Function):
    """Strided conv, filter_size == stride: out[p] = sum_o W[o]^T x[child(p, o)] (§8(a) a7)."""

    @staticmethod
    def forward(ctx, x, weight, rules, n_coarse, parts=None):
        """parts: BnParts for the forward sums of the output, for the BatchNorm it feeds (SubmanifoldConvFunction)."""
        _check_feats(x)
        K, _, cin, cout = weight.shape
        cin_p, cout_p = _pad16(cin), _pad16(cout)
        xp = _pad_cols(x.contiguous(), cin_p)
        wp = _pad_weight(weight.reshape(K, cin, cout), cin_p, cout_p)
        epi = None
        if parts is not None and cout_p == cout and parts.C == cout and \
                bn_epi_ok(rules, n_coarse, cin_p, cout_p, K):
            epi = (parts, None, None, 0.0)
        out = conv_tile(xp, wp, K, 2, cout_p, rules, n_coarse, "conv_fwd", 2.0 * x.size(0) * cin * cout, epi=epi)
        ctx.save_for_backward(xp, wp)
        ctx.rules, ctx.dims = rules, (cin, cout)
        return out if cout_p == cout else out[:, :cout].contiguous()

    @staticmethod
    def backward(ctx, gout):
        xp, wp = ctx.saved_tensors
        rules, (cin, cout) = ctx.rules, ctx.dims
        K, cin_p, cout_p = wp.shape
        g = _pad_cols(gout.contiguous(), cout_p)
        rules.note_use("pairs", 0, 0)
        p = rules.pairs
        dx = dw = None
        join = None
        if ctx.needs_input_grad[1]:
            flops = 2.0 * xp.size(0) * cin * cout  # one rule per fine row
            dwp = None
            if STRIDED_WGRAD_CHUNK:
                # the chunk weight gradient over the child map: tiles of 128 coarse rows (dy), their children's
                # distinct fine rows (x) staged once per tile (round 6)
                rules.note_use("wgrad", cin_p, cout_p)
                if int(_lib.query("msp_wgrad_chunk_preferred", _lib.I64(g.size(0)), K, cin_p, cout_p)) and \
                        rules.wgrad_index(wait=True) is not None:
                    dwp, join = _on_side(xp, g.size(0), lambda: conv_wgrad_chunk(xp, g, rules, K, "wgrad_strided",
                                                                                flops))
            if dwp is None:
                dwp, join = conv_wgrad_async(xp, g, p, p.pair_in, p.pair_out, K, flops, "wgrad_strided")
            dw = dwp[:, :cin, :cout].reshape(K, 1, cin, cout)
        if ctx.needs_input_grad[0]:
            # dx[fine] = W[o] g[parent]: src = coarse (pair_out), dst = fine (pair_in)
            dxp = conv_pairs(g, wp, K, cin_p, p, p.pair_out, p.pair_in, xp.size(0), "conv_bwd_data",
                             2.0 * p.total * cin * cout)
            dx = dxp if cin_p == cin else dxp[:, :cin]
        if join is not None:
            join()
        return dx, dw, None, None, None


class DeconvolutionFunction(torch.autograd.Function):
    """Transpose of ConvolutionFunction on the same rules (§8(a) a8):
    out[fine] = W[o]^T x[parent(fine)]."""

    @staticmethod
    def forward(ctx, x, weight, rules, n_fine, link=None):
        """link: BnLink of the BatchNorm whose output x is (its backward sums from the backward-data's epilogue)."""
        _check_feats(x)
        K, _, cin, cout = weight.shape
        cin_p, cout_p = _pad16(cin), _pad16(cout)
        xp = _pad_cols(x.contiguous(), cin_p)
        wp = _pad_weight(weight.reshape(K, cin, cout), cin_p, cout_p)
        wt = wp.transpose(1, 2).contiguous()
        rules.note_use("pairs", 0, 0)  # the forward and both backward passes run on the pair lists
        p = rules.pairs
        out = conv_pairs(xp, wt, K, cout_p, p, p.pair_out, p.pair_in, n_fine, "deconv_fwd", 2.0 * p.total * cin * cout)
        ctx.save_for_backward(xp, wp)
        ctx.rules, ctx.dims = rules, (cin, cout)
        ctx.link = link if (link is not None and cin_p == cin) else None
        return out if cout_p == cout else out[:, :cout].contiguous()

    @staticmethod
    def backward(ctx, gout):
        xp, wp = ctx.saved_tensors
        rules, (cin, cout) = ctx.rules, ctx.dims
        K, cin_p, cout_p = wp.shape
        g = _pad_cols(gout.contiguous(), cout_p)
        p = rules.pairs
        dx = dw = None
        join = None
        if ctx.needs_input_grad[1]:
            flops = 2.0 * g.size(0) * cin * cout  # one rule per fine row
            dwp = None
            if STRIDED_WGRAD_CHUNK:
                # the chunk form over the child map with the roles swapped (the coarse input rows are the tiles'
                # own rows, the fine output gradients the gathered ones): it gives dW^T per offset (round 6)
                rules.note_use("wgrad", cout_p, cin_p)
                if int(_lib.query("msp_wgrad_chunk_preferred", _lib.I64(xp.size(0)), K, cout_p, cin_p)) and \
                        rules.wgrad_index(wait=True) is not None:
                    dwp, join = _on_side(xp, xp.size(0), lambda: conv_wgrad_chunk(g, xp, rules, K, "wgrad_deconv",
                                                                                 flops).transpose(1, 2))
            if dwp is None:
                dwp, join = conv_wgrad_async(xp, g, p, p.pair_out, p.pair_in, K, flops, "wgrad_deconv")
            dw = dwp[:, :cin, :cout].reshape(K, 1, cin, cout)
        if ctx.needs_input_grad[0]:
            V = xp.size(0)
            link, epi = ctx.link, None
            if link is not None and link.x is not None and bn_epi_ok(rules, V, cout_p, cin_p, K):
                epi = (BnParts(cin_p, V, g.device), link.x, link.stats, link.leak)
            dxp = conv_tile(g, wp, K, 0, cin_p, rules, V, "deconv_bwd_data",
                            2.0 * g.size(0) * cin * cout, epi=epi)
            if epi is not None:
                link.bwd = (dxp, epi[0])
            dx = dxp if cin_p == cin else dxp[:, :cin]
        if join is not None:
            join()
        ctx.link = None
        return dx, dw, None, None, None


# ------------------------------------------------------------------ network-in-network
_ARANGE = {}  # device index -> int32 arange, grown on demand (identity pair lists)


class _IdentityPairs:
    """Pair lists of the per-site linear map: row i -> row i (one 'offset').
    Built with device fills only (no host-to-device copy that would
    synchronise the host inside backward)."""

    def __init__(self, n, device):
        self.total = int(n)
        self.off_start = torch.zeros(2, dtype=torch.int64, device=device)
        self.off_start[1:].fill_(self.total)
        ar = _ARANGE.get(device.index)
        if ar is None or ar.numel() < max(n, 1):
            ar = _ARANGE[device.index] = torch.arange(max(n, 1 << 16), dtype=torch.int32, device=device)
        self.pair = ar[:max(n, 1)]


NIN_MAX_K = 1024  # msp_nin_gemm_ok: the split image of B's K rows must fit the kernel's LDS budget


def _aligned16(t):
    """t itself when its data is 16-byte aligned (msp_nin_gemm's float4 loads), else an aligned copy."""
    return t if t.data_ptr() % 16 == 0 else t.clone()


def nin_gemm(a, b, kind="nin", keep_pad=False):
    """a[M][K] @ b[K][N] on msp_nin_gemm (HBM-bound tall-skinny product: fp32 MFMA from 2^18 rows, split-bf16
    MFMA below); channel counts that are not multiples of 16 are zero-padded around the call (keep_pad: the
    [M][pad16(N)] result is returned as is, its last columns zero).  Any nIn works (SCN's NetworkInNetwork takes
    any): K beyond the kernel's 1024 is contracted in 1024-deep slices whose products are added in slice order;
    operands that are not 16-byte aligned (a view with an odd storage offset) are copied first."""
    M, K = a.shape
    N = b.size(1)
    Kp, Np = _pad16(K), _pad16(N)
    if Kp != K:
        a, b = _pad_cols(a.contiguous(), Kp), torch.cat([b, b.new_zeros(Kp - K, N)])
    if Np != N:
        b = _pad_cols(b, Np)
    a, b = _aligned16(a.contiguous()), _aligned16(b.contiguous())
    flops, nbytes = 2.0 * M * K * N, 4 * (M * K + M * N + K * N)
    out = None
    for k0 in range(0, Kp, NIN_MAX_K):
        k1 = min(Kp, k0 + NIN_MAX_K)
        ak = a if (k0 == 0 and k1 == Kp) else a[:, k0:k1].contiguous()
        bk = b if (k0 == 0 and k1 == Kp) else b[k0:k1].contiguous()
        kk = k1 - k0
        part = torch.empty((max(M, 1), Np), dtype=torch.float32, device=a.device)
        wsb = int(_lib.query("msp_nin_gemm_workspace_size", kk, Np))
        ws = torch.empty(max(wsb // 4, 1), dtype=torch.float32, device=a.device)
        form = "/f32" if int(_lib.query("msp_nin_gemm_form", _lib.I64(M), kk, Np)) == 1 else "/x6"
        _record(kind + form, flops * kk / Kp, lambda: call("msp_nin_gemm", ptr(ak), M, kk, ptr(bk), Np, ptr(part),
                                                           ptr(ws), wsb, _stream(a)), nbytes * kk // Kp)
        out = part if out is None else out.add_(part)
    out = out[:M]
    return out if (Np == N or keep_pad) else out[:, :N].contiguous()


class NetworkInNetworkFunction(torch.autograd.Function):
    """out = x W (§8(a) a11).  Forward and backward-data on msp_nin_gemm (W, then W^T); the weight gradient
    x^T dy (a contraction over all V rows) runs on msp_conv_wgrad as a one-offset convolution with identity
    pairs."""

    @staticmethod
    def forward(ctx, x, weight):
        _check_feats(x)
        x = x.contiguous()
        ctx.save_for_backward(x, weight)
        return nin_gemm(x, weight, kind="nin_fwd")

    @staticmethod
    def backward(ctx, gout):
        x, weight = ctx.saved_tensors
        g = gout.contiguous()
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = nin_gemm(g, weight.t(), kind="nin_bwd_data")
        if ctx.needs_input_grad[1]:
            cin, cout = weight.shape
            cin_p, cout_p = _pad16(cin), _pad16(cout)
            p = _IdentityPairs(x.size(0), x.device)
            dw = conv_wgrad(_pad_cols(x, cin_p), _pad_cols(g, cout_p), p, p.pair, p.pair, 1, "nin_wgrad",
                            2.0 * p.total * cin * cout)[0, :cin, :cout]
        return dx, dw


# ------------------------------------------------------------------ batch norm
def _bn_partial_buf(V, C, device):
    P = int(_lib.query("msp_bn_partials", _lib.I64(V), C))
    return torch.empty((P + 1) * 2 * C, dtype=torch.float64, device=device)


def _bn_fwd(x, weight, bias, running_mean, running_var, eps, momentum, leak, train, partial):
    """y, stats of BN + (leaky) ReLU; `partial` = the msp_bn_stats partials of
    x when a residual join already produced them (msp_add_bn_stats), else None."""
    V, C = x.shape
    s = _stream(x)
    stats = torch.empty((5, C), dtype=torch.float32, device=x.device)
    y = torch.empty_like(x)

    def run(partial=partial):
        if isinstance(partial, BnParts):  # the producing convolution's epilogue sums (channel-major)
            call("msp_bn_finalize_cm", ptr(partial.buf), partial.P, V, C, float(eps), float(momentum), int(train),
                 ptr(running_mean), ptr(running_var), ptr(weight), ptr(bias), ptr(stats), s)
        else:
            if partial is None:
                partial = _bn_partial_buf(V, C, x.device)
                if train:
                    call("msp_bn_stats", ptr(x), V, C, ptr(partial), s)
            call("msp_bn_finalize", ptr(partial), V, C, float(eps), float(momentum), int(train),
                 ptr(running_mean), ptr(running_var), ptr(weight), ptr(bias), ptr(stats), s)
        call("msp_bn_apply", ptr(x), V, C, ptr(stats), float(leak), ptr(y), s)
    # compulsory bytes: statistics pass (read x) unless a join produced them, apply (read x, write y)
    _record(_shape("bn_fwd/hbm", C, C, V), 0, run, 4 * V * C * (3 if (partial is None and train) else 2))
    return y, stats


def _bn_bwd(x, weight, stats, cfg, gy, addend, link=None):
    """dx (+ addend, fused), dweight, dbias.  link: the BnLink whose consumer's backward-data may have left this
    BN's backward sums (used when gy is exactly the gradient that call returned)."""
    leak, train, has_w, has_b = cfg
    gy = gy.contiguous()
    V, C = x.shape
    s = _stream(x)
    parts = None
    if link is not None and link.bwd is not None:
        d, p = link.bwd
        link.bwd = None
        if p.written and d.data_ptr() == gy.data_ptr() and tuple(d.shape) == tuple(gy.shape) and p.C == C:
            parts = p
    dx = torch.empty_like(x)
    dw = torch.empty(C, dtype=torch.float32, device=x.device)
    db = torch.empty(C, dtype=torch.float32, device=x.device)
    add = ptr(addend) if addend is not None else None
    wp = ptr(weight) if has_w else None
    if parts is not None:
        # compulsory bytes: apply only (read x, dy [, shortcut grad], write dx); the sums came with dy
        _record(_shape("bn_bwd/hbm", C, C, V), 0, lambda: call(
            "msp_bn_bwd_apply_cm", ptr(x), ptr(gy), V, C, ptr(parts.buf), parts.P, ptr(stats), wp, leak, train, add,
            ptr(dx), ptr(dw), ptr(db), s), 4 * V * C * (3 + (addend is not None)))
        return dx, (dw if has_w else None), (db if has_b else None)
    partial = _bn_partial_buf(V, C, x.device)

    def run():
        call("msp_bn_bwd_stats", ptr(x), ptr(gy), V, C, ptr(stats), leak, ptr(partial), s)
        call("msp_bn_bwd_apply_add", ptr(x), ptr(gy), V, C, ptr(partial), ptr(stats), wp, leak, train, add, ptr(dx),
             ptr(dw), ptr(db), s)
    # compulsory bytes: statistics pass (read x, dy), apply (read x, dy [, shortcut grad], write dx)
    _record(_shape("bn_bwd/hbm", C, C, V), 0, run, 4 * V * C * (5 + (addend is not None)))
    return dx, (dw if has_w else None), (db if has_b else None)


def _link(link, x, stats, train):
    """The BnLink of a training-mode BN forward, filled with its input and statistics (else None)."""
    if link is None or not train:
        return None
    link.x, link.stats = x, stats
    return link


class BatchNormFunction(torch.autograd.Function):
    """BatchNormalization + (leaky) ReLU; stats[5][C] as in include/mi3dsparse.h.
    `partial`: precomputed batch-statistic partials of x (ResidualJoinFunction)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, leak, train, partial=None,
                link=None):
        _check_feats(x)
        x = x.contiguous()
        y, stats = _bn_fwd(x, weight, bias, running_mean, running_var, eps, momentum, leak, train, partial)
        ctx.save_for_backward(x, weight, stats)
        ctx.cfg = (float(leak), int(train), weight is not None, bias is not None)
        ctx.link = _link(link, x, stats, train)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, stats = ctx.saved_tensors
        dx, dw, db = _bn_bwd(x, weight, stats, ctx.cfg, gy, None, ctx.link)
        ctx.link = None
        return dx, dw, db, None, None, None, None, None, None, None, None


class BatchNormForkFunction(torch.autograd.Function):
    """x -> (BN-ReLU(x), x): the residual fork of SCN's ConcatTable(shortcut,
    Sequential(BatchNorm..., ...)) (networkArchitectures.py blocks, UNet skip
    joins).  The second output is x itself (a view) for the shortcut; the
    backward adds the shortcut's gradient of x inside the BN backward kernel
    (msp_bn_bwd_apply_add) instead of autograd's separate accumulation add."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, leak, train, partial=None,
                link=None):
        _check_feats(x)
        x = x.contiguous()
        ctx.set_materialize_grads(False)
        y, stats = _bn_fwd(x, weight, bias, running_mean, running_var, eps, momentum, leak, train, partial)
        ctx.save_for_backward(x, weight, stats)
        ctx.cfg = (float(leak), int(train), weight is not None, bias is not None)
        ctx.link = _link(link, x, stats, train)
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, gy, gx):
        x, weight, stats = ctx.saved_tensors
        link, ctx.link = ctx.link, None
        if gy is None:
            return gx, None, None, None, None, None, None, None, None, None, None
        if gx is not None:
            gx = gx.contiguous()
        dx, dw, db = _bn_bwd(x, weight, stats, ctx.cfg, gy, gx, link)
        return dx, dw, db, None, None, None, None, None, None, None, None


def _bn_bwd_split(x, weight, stats, cfg, gy, addend, ca, need_a, need_b):
    """_bn_bwd with dx written as its two column blocks [V][ca], [V][C - ca] (msp_bn_bwd_apply_split): the
    gradients of the JoinTable inputs that x joined, with no split pass.  Returns (ga, gb, dweight, dbias)."""
    leak, train, has_w, has_b = cfg
    gy = gy.contiguous()
    V, C = x.shape
    s = _stream(x)
    ga = torch.empty((V, ca), dtype=torch.float32, device=x.device)
    gb = torch.empty((V, C - ca), dtype=torch.float32, device=x.device)
    dw = torch.empty(C, dtype=torch.float32, device=x.device)
    db = torch.empty(C, dtype=torch.float32, device=x.device)
    partial = _bn_partial_buf(V, C, x.device)
    add = ptr(addend) if addend is not None else None

    def run():
        call("msp_bn_bwd_stats", ptr(x), ptr(gy), V, C, ptr(stats), leak, ptr(partial), s)
        call("msp_bn_bwd_apply_split", ptr(x), ptr(gy), V, C, ptr(partial), ptr(stats),
             ptr(weight) if has_w else None, leak, train, add, ca, ptr(ga), ptr(gb), ptr(dw), ptr(db), s)
    # compulsory bytes: statistics pass (read x, dy), apply (read x, dy [, shortcut grad], write dx's two blocks)
    _record(_shape("bn_bwd/hbm", C, C, V), 0, run, 4 * V * C * (5 + (addend is not None)))
    return (ga if need_a else None), (gb if need_b else None), (dw if has_w else None), (db if has_b else None)


# The UNet decoder's JoinTable -> BatchNormalization: the BN's backward writes the join inputs' gradients itself
# (BatchNormJoinFunction) instead of a [V][C] dx that JoinFunction's backward then splits (msp_split_cols: one read
# and one write of V x C floats per join, 0.26 ms/step at C3).  False: JoinFunction's split, as before.
FUSE_JOIN_SPLIT = True


class BatchNormJoinFunction(torch.autograd.Function):
    """BatchNormFunction / BatchNormForkFunction (fork = True: the second output is x for the shortcut, whose
    gradient is added inside the backward) over the output x = [a | b] of a JoinTable.  x comes in detached (the
    join's forward already ran and left its statistics partials); a and b carry the gradient: the backward
    writes d[a | b] as its two column blocks (msp_bn_bwd_apply_split), so the join's split pass is not needed.
    The join's own autograd node receives no gradient from here; any other consumer of the joined tensor still
    back-propagates through it (JoinFunction's split), and autograd adds the two contributions to a and b."""

    @staticmethod
    def forward(ctx, x, a, b, fork, weight, bias, running_mean, running_var, eps, momentum, leak, train,
                partial=None, link=None):
        _check_feats(x)
        if x.size(1) != a.size(1) + b.size(1) or x.size(0) != a.size(0):
            raise ValueError(f"BatchNormJoinFunction: x {tuple(x.shape)} is not the join of {tuple(a.shape)} and "
                             f"{tuple(b.shape)}")
        x = x.contiguous()
        ctx.set_materialize_grads(False)
        y, stats = _bn_fwd(x, weight, bias, running_mean, running_var, eps, momentum, leak, train, partial)
        ctx.save_for_backward(x, weight, stats)
        ctx.cfg = (float(leak), int(train), weight is not None, bias is not None)
        ctx.ca = a.size(1)
        ctx.link = _link(link, x, stats, train)
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, gy, gx):
        x, weight, stats = ctx.saved_tensors
        link, ctx.link = ctx.link, None
        if link is not None:
            link.bwd = None  # a consumer's epilogue sums are not used on this path
        need_a, need_b = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        none = (None,) * 10
        if gy is None:
            if gx is None:
                return (None, None, None) + none + (None,)
            gx = gx.contiguous()
            V, C = gx.shape
            ga = torch.empty((V, ctx.ca), dtype=torch.float32, device=gx.device) if need_a else None
            gb = torch.empty((V, C - ctx.ca), dtype=torch.float32, device=gx.device) if need_b else None
            if ga is not None or gb is not None:
                call("msp_split_cols", ptr(gx), V, ctx.ca, C - ctx.ca, ptr(ga), ptr(gb), _stream(gx))
            return (None, ga, gb) + none + (None,)
        if gx is not None:
            gx = gx.contiguous()
        ga, gb, dw, db = _bn_bwd_split(x, weight, stats, ctx.cfg, gy, gx, ctx.ca, need_a, need_b)
        return (None, ga, gb, None, dw, db) + (None,) * 8


class ResidualJoinFunction(torch.autograd.Function):
    """a + b (SCN AddTable of a residual block) fused with the batch-statistic
    partials of the sum (msp_add_bn_stats): the next BatchNormalization, which
    every residual join in the UNet/FCN builders feeds, skips its own pass
    over the sum.  Returns (sum, partials); the partials carry no gradient."""

    @staticmethod
    def forward(ctx, a, b):
        _check_feats(a)
        _check_feats(b)
        a, b = a.contiguous(), b.contiguous()
        V, C = a.shape
        out = torch.empty_like(a)
        partial = _bn_partial_buf(V, C, a.device)
        _record(_shape("bn_join/hbm", C, C, V), 0, lambda: call("msp_add_bn_stats", ptr(a), ptr(b), V, C, ptr(out), ptr(partial),
                                                _stream(a)), 12 * V * C)
        ctx.mark_non_differentiable(partial)
        ctx.set_materialize_grads(False)  # no zero-filled fp64 "gradient" of the partials per join
        return out, partial

    @staticmethod
    def backward(ctx, g, _gp):
        return g, g


class JoinFunction(torch.autograd.Function):
    """[a | b] along channels (SCN JoinTable of the UNet / FCN skip joins: identity branch first, §8(a) a12) on
    msp_join_cols, with the batch-statistic partials of the result when `stats` (the BatchNormalization the
    join feeds then skips its own pass over it, as after a residual join); backward splits the gradient in one
    pass (msp_split_cols).  Returns (joined, partials or None)."""

    @staticmethod
    def forward(ctx, a, b, stats):
        _check_feats(a)
        _check_feats(b)
        if a.dim() != 2 or b.dim() != 2 or b.size(0) != a.size(0):
            raise ValueError(f"JoinTable: inputs must be [V, C] with the same row count, got {tuple(a.shape)} and "
                             f"{tuple(b.shape)}")
        if a.device != b.device:
            raise ValueError(f"JoinTable: inputs on different devices ({a.device} and {b.device})")
        a, b = a.contiguous(), b.contiguous()
        V, ca = a.shape
        cb = b.size(1)
        C = ca + cb
        out = torch.empty((V, C), dtype=torch.float32, device=a.device)
        partial = _bn_partial_buf(V, C, a.device) if stats else None
        _record(_shape("bn_join/hbm", C, C, V), 0, lambda: call(
            "msp_join_cols", ptr(a), ca, ptr(b), cb, V, ptr(out), ptr(partial), _stream(a)), 8 * V * C)
        ctx.dims = (ca, cb)
        ctx.set_materialize_grads(False)
        if partial is not None:
            ctx.mark_non_differentiable(partial)
        return out, partial

    @staticmethod
    def backward(ctx, g, _gp):
        if g is None:
            return None, None, None
        ca, cb = ctx.dims
        g = g.contiguous()
        V = g.size(0)
        ga = torch.empty((V, ca), dtype=torch.float32, device=g.device) if ctx.needs_input_grad[0] else None
        gb = torch.empty((V, cb), dtype=torch.float32, device=g.device) if ctx.needs_input_grad[1] else None
        if ga is not None or gb is not None:
            call("msp_split_cols", ptr(g), V, ca, cb, ptr(ga), ptr(gb), _stream(g))
        return ga, gb, None


# ------------------------------------------------------------------ input / output / pooling
class InputLayerFunction(torch.autograd.Function):
    """mode 3 (sum) / 4 (mean) point -> voxel reduction (§8(a) a4)."""

    @staticmethod
    def forward(ctx, feats, rules, n_vox, mode):
        _check_feats(feats)
        feats = feats.contiguous()
        C = feats.size(1)
        s = _stream(feats)
        out = torch.empty((max(n_vox, 1), C), dtype=torch.float32, device=feats.device)
        if n_vox:
            if mode == 4:
                call("msp_input_avg_fwd", ptr(feats), C, ptr(rules.perm), ptr(rules.vstart), n_vox, ptr(out), s)
            else:
                call("msp_output_bwd", ptr(feats), C, ptr(rules.perm), ptr(rules.vstart), n_vox, ptr(out), s)
        ctx.rules, ctx.mode, ctx.n = rules, mode, feats.size(0)
        return out[:n_vox]

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        rules = ctx.rules
        C = g.size(1)
        df = torch.empty((max(ctx.n, 1), C), dtype=torch.float32, device=g.device)
        if ctx.n:
            if ctx.mode == 4:
                call("msp_input_avg_bwd", ptr(g), C, ptr(rules.p2v), ptr(rules.vstart), ctx.n, ptr(df), _stream(g))
            else:
                call("msp_output_fwd", ptr(g), C, ptr(rules.p2v), ctx.n, ptr(df), _stream(g))
        return df[:ctx.n], None, None, None


class OutputLayerFunction(torch.autograd.Function):
    """voxel -> point gather through the InputLayer map (§8(a) a14)."""

    @staticmethod
    def forward(ctx, x, rules):
        _check_feats(x)
        x = x.contiguous()
        C = x.size(1)
        out = torch.empty((max(rules.n_points, 1), C), dtype=torch.float32, device=x.device)
        if rules.n_points:
            call("msp_output_fwd", ptr(x), C, ptr(rules.p2v), rules.n_points, ptr(out), _stream(x))
        ctx.rules, ctx.V = rules, x.size(0)
        return out[:rules.n_points]

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        rules = ctx.rules
        C = g.size(1)
        din = torch.empty((max(ctx.V, 1), C), dtype=torch.float32, device=g.device)
        if ctx.V:
            call("msp_output_bwd", ptr(g), C, ptr(rules.perm), ptr(rules.vstart), ctx.V, ptr(din), _stream(g))
        return din[:ctx.V], None


class SceneMeanFunction(torch.autograd.Function):
    """Fused OutputLayer + per-scene mean over the points (SURVEY.md §8(f)
    rank 2; models/SparseConvNet.py:20-26) from the level-0 voxel rows:
    out[b] = sum_v cnt_v feat[v] / n_b without the (N, C) per-point tensor."""

    @staticmethod
    def forward(ctx, x, level, rules, B):
        _check_feats(x)
        x = x.contiguous()
        V, C = x.shape
        dev = x.device
        vscene = torch.empty(B + 1, dtype=torch.int64, device=dev)
        npts = torch.empty(B, dtype=torch.int64, device=dev)
        out = torch.empty((B, C), dtype=torch.float32, device=dev)
        wsb = int(_lib.query("msp_scene_mean_workspace_size", _lib.I64(V), B, C))
        ws = torch.empty(max(wsb, 8), dtype=torch.uint8, device=dev)
        shift = 3 * level.log2
        call("msp_scene_mean_fwd", ptr(x), C, ptr(level.keys), V, shift, ptr(rules.vstart), B, ptr(vscene),
             ptr(npts), ptr(out), ptr(ws), wsb, _stream(x))
        ctx.level, ctx.rules, ctx.V, ctx.shift = level, rules, V, shift
        ctx.save_for_backward(npts)
        ctx.mark_non_differentiable(npts)
        ctx.set_materialize_grads(False)
        return out, npts

    @staticmethod
    def backward(ctx, g, _gn):
        (npts,) = ctx.saved_tensors
        if g is None:
            return None, None, None, None
        g = g.contiguous()
        C = g.size(1)
        dx = torch.empty((max(ctx.V, 1), C), dtype=torch.float32, device=g.device)
        call("msp_scene_mean_bwd", ptr(g), C, ptr(ctx.level.keys), ctx.V, ctx.shift, ptr(ctx.rules.vstart),
             ptr(npts), ptr(dx), _stream(g))
        return dx[:ctx.V], None, None, None


class PointLogitsFunction(torch.autograd.Function):
    """Per-point logits of the head's Linear without the (N, C) per-point features (the
    eval half; models/MultiLabelContrastive.py:43-45 `self.linear(self.pc_encoder(x))`, :84-101, train.py:106):
    logits[p] = W x[v(p)] + b.  The Linear commutes with the OutputLayer's gather, so it runs on the level-0
    voxel rows ((V, C) @ W^T on msp_nin_gemm) and each point gathers its voxel's n_out columns plus the bias
    (msp_point_rows_bias).  Backward: the points' gradients summed per voxel (msp_output_bwd, fixed order),
    dW from those sums (msp_conv_wgrad, identity pairs), dx = g_v W (msp_nin_gemm), db = column sums."""

    @staticmethod
    def forward(ctx, x, weight, bias, rules):
        _check_feats(x)
        x = x.contiguous()
        V, C = x.shape
        n_out = weight.size(0)
        if weight.size(1) != C:
            raise ValueError(f"PointLogits: Linear({weight.size(1)}, {n_out}) on {C} channels")
        vl = nin_gemm(x, weight.t(), kind="logits_fwd", keep_pad=True)  # (V, pad16(n_out))
        out = torch.empty((max(rules.n_points, 1), n_out), dtype=torch.float32, device=x.device)
        if rules.n_points:
            call("msp_point_rows_bias", ptr(vl), vl.size(1), n_out, ptr(bias.contiguous()) if bias is not None
                 else None, ptr(rules.p2v), rules.n_points, ptr(out), _stream(x))
        ctx.save_for_backward(x, weight)
        ctx.rules, ctx.has_bias = rules, bias is not None
        return out[:rules.n_points]

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        rules = ctx.rules
        V, C = x.shape
        n_out = weight.size(0)
        g = g.contiguous()
        gv = torch.empty((max(V, 1), n_out), dtype=torch.float32, device=g.device)
        if V:
            call("msp_output_bwd", ptr(g), n_out, ptr(rules.perm), ptr(rules.vstart), V, ptr(gv), _stream(g))
        gv = gv[:V]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = nin_gemm(gv, weight, kind="logits_bwd_data")
        if ctx.needs_input_grad[1]:
            cin_p, cout_p = _pad16(C), _pad16(n_out)
            p = _IdentityPairs(V, x.device)
            dw = conv_wgrad(_pad_cols(x, cin_p), _pad_cols(gv, cout_p), p, p.pair, p.pair, 1, "logits_wgrad",
                            2.0 * V * C * n_out)[0, :C, :n_out].t()
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = gv.sum(0)
        return dx, dw, db, None


def index_add_rows(store, ids, src):
    """store.index_add_(0, ids, src) on the device, bit-equal to the serial CPU loop for any ids
    (msp_index_add_rows); ids outside [0, len(store)) raise IndexError like torch's (one host read)."""
    _check_feats(store)
    _check_feats(src)
    if store.dim() != 2 or src.dim() != 2 or src.size(1) != store.size(1) or ids.numel() != src.size(0):
        raise ValueError(f"index_add_rows: store {tuple(store.shape)}, ids {tuple(ids.shape)}, src {tuple(src.shape)}")
    if not store.is_contiguous():
        raise ValueError("index_add_rows: store must be contiguous (it is updated in place)")
    n = ids.numel()
    if n == 0:
        return store
    ids = ids.to(device=store.device, dtype=torch.int64).contiguous()
    lo, hi = torch.aminmax(ids)
    if int(lo) < 0 or int(hi) >= store.size(0):
        raise IndexError(f"index_add_rows: index out of range [0, {store.size(0)}) (min {int(lo)}, max {int(hi)})")
    src = src.contiguous()
    wsb = int(_lib.query("msp_index_add_workspace_size", n, store.size(0)))
    ws = torch.empty(max(wsb, 8), dtype=torch.uint8, device=store.device)
    call("msp_index_add_rows", ptr(store), store.size(0), store.size(1), ptr(ids), ptr(src), n, ptr(ws), wsb,
         _stream(store))
    return store


class UnPoolingFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rules, n_fine):
        _check_feats(x)
        x = x.contiguous()
        C = x.size(1)
        out = torch.empty((max(n_fine, 1), C), dtype=torch.float32, device=x.device)
        if n_fine:
            call("msp_unpool_fwd", ptr(x), C, ptr(rules.parent_of), n_fine, ptr(out), _stream(x))
        ctx.rules, ctx.Vc = rules, x.size(0)
        return out[:n_fine]

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        C = g.size(1)
        din = torch.empty((max(ctx.Vc, 1), C), dtype=torch.float32, device=g.device)
        if ctx.Vc:
            call("msp_unpool_bwd", ptr(g), C, ptr(ctx.rules.child_start), ctx.Vc, ptr(din), _stream(g))
        return din[:ctx.Vc], None, None


class MaxPoolingFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rules, n_coarse):
        _check_feats(x)
        x = x.contiguous()
        C = x.size(1)
        out = torch.empty((max(n_coarse, 1), C), dtype=torch.float32, device=x.device)
        arg = torch.empty((max(n_coarse, 1), C), dtype=torch.int32, device=x.device)
        if n_coarse:
            call("msp_maxpool_fwd", ptr(x), C, ptr(rules.child_start), n_coarse, ptr(out), ptr(arg), _stream(x))
        ctx.save_for_backward(arg)
        ctx.Vf, ctx.Vc = x.size(0), n_coarse
        return out[:n_coarse]

    @staticmethod
    def backward(ctx, g):
        (arg,) = ctx.saved_tensors
        g = g.contiguous()
        C = g.size(1)
        din = torch.zeros((max(ctx.Vf, 1), C), dtype=torch.float32, device=g.device)
        if ctx.Vc:
            call("msp_maxpool_bwd", ptr(g), C, ptr(arg), ctx.Vc, ptr(din), _stream(g))
        return din[:ctx.Vf], None, None
