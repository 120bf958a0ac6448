"""Per-forward sparse metadata, built on the device.

SCN keeps one `Metadata` per InputLayer call: a hash grid per spatial size and
rulebooks cached per (operation, spatial size), built on the host
(SURVEY.md §3.1, §8(a) a4/a5/a7).  This class keeps the same caching contract
-- one `Level` per spatial size, one submanifold rulebook per filter size, one
strided map per stride -- but every structure lives in HBM and is produced by
the kernels of libmi3dsparse:

  Level            sorted Morton keys of the active sites (V rows)
  SubmRules        offset-major neighbour map nbr[K][V], the output-tile
                   rulebook for msp_conv_tile and per-offset pair lists
                   for the weight gradient
  DownRules        parent of every fine site, child runs per coarse site,
                   child map down[K][Vc] + its tile rulebook and pair lists

The only device->host reads are the counts that size the next allocation
(V per level, rulebook chunk totals, per-offset list starts).  A replay (the
prefetch of the next batch) defers the rulebook counts and reads them together:
one read per coarsening (its V, with every count queued before it) and one at
the end, instead of one per rulebook.
"""
from __future__ import annotations

import math
import os
import threading

import torch

from . import _lib
from ._lib import I64, call, ptr, query

CHUNK = 16      # MSP_CHUNK


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 8), dtype=torch.uint8, device=device)


def _log2_ceil(n: int) -> int:
    return max(1, int(math.ceil(math.log2(max(2, int(n))))))


class _Deferred:
    """The count reads of one replay, batched.  read(t, fn) queues fn(values of the int64 device tensor t);
    then(fn) queues work that needs every queued read applied; flush() applies them with one device->host copy
    per round (reads first, then the dependent work, until neither is left), on the stream the build runs on --
    so a flush forced from elsewhere still orders the copy after the counting kernels."""

    def __init__(self, stream):
        self.stream = stream
        self.reads, self.after = [], []

    def read(self, t, fn):
        self.reads.append((t, fn))

    def then(self, fn):
        self.after.append(fn)

    def flush(self):
        import contextlib
        with torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext():
            while self.reads or self.after:
                if self.reads:
                    reads, self.reads = self.reads, []
                    flat = _host(reads[0][0] if len(reads) == 1 else torch.cat([t.reshape(-1) for t, _ in reads]))
                    k = 0
                    for t, fn in reads:
                        fn([int(v) for v in flat[k:k + t.numel()]])
                        k += t.numel()
                else:
                    after, self.after = self.after, []
                    for fn in after:
                        fn()


_TLS = threading.local()  # .defer: this thread's replay in progress (a prefetch may build on a worker thread)
# MSP_DEFER_READS=0: a replay reads every count where it is taken, as an inline build does (A/B switch)
DEFER_READS = os.environ.get("MSP_DEFER_READS", "1") != "0"


# MSP_LOCAL_CHUNK_INDEX=0: the chunk weight gradient's index always from the 128-row tile rulebook (A/B switch;
# SubmRules._local_chunk_index)
LOCAL_CHUNK_INDEX = os.environ.get("MSP_LOCAL_CHUNK_INDEX", "1") != "0"


# MSP_PINNED_READS=0: count reads as Tensor.cpu() (A/B switch; see _host)
PINNED_READS = os.environ.get("MSP_PINNED_READS", "1") != "0"


READ_STATS = None  # [seconds, reads]: host time spent in count reads (bench.py BENCH_HOST_TIMING), None: off


def _host(t):
    if READ_STATS is not None:
        import time
        t0 = time.perf_counter()
        v = _host_read(t)
        READ_STATS[0] += time.perf_counter() - t0
        READ_STATS[1] += 1
        return v
    return _host_read(t)


def _host_read(t):
    """Values of a device tensor as a Python list.  The copy goes into pinned host memory without blocking and
    the host then waits on an event of the current stream alone (a blocking copy to pageable memory may wait for
    more than that stream's work).  Both waits let go of the GIL: a prefetch on a worker thread does not hold up
    the thread capturing a step."""
    if not PINNED_READS or t.device.type != "cuda":
        return t.cpu().tolist()
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    ev.synchronize()
    return h.tolist()


def _defer():
    return getattr(_TLS, "defer", None)


class _PendingIndex:
    """SubmRules._wchunk while a replay's count reads are still queued (wgrad_index decides once they are read).
    Not an index: consumers call wgrad_index(wait=True), which flushes the replay's reads first."""

    def __repr__(self):
        return "<weight-gradient index pending>"


_PENDING = _PendingIndex()


def _later(t, fn):
    """fn(values of the int64 device tensor t): now, or at the next flush of the replay in progress."""
    d = _defer()
    if d is None:
        fn([int(v) for v in _host(t)])
    else:
        d.read(t, fn)


def _resolve():
    d = _defer()
    if d is not None:
        d.flush()


def tile_rulebook(m, K, n, device, s, tile_rows=64):
    """Output-tile rulebook of an offset-major map m[K][n] (two passes:
    count, then fill, sized by one host read of the chunk total -- deferred in a replay: the
    dict has its chunk arrays once the replay's counts are read)."""
    tr = int(tile_rows)
    n_tiles = (n + tr - 1) // tr
    # tile_start[n_tiles + 1] = largest chunk count of one tile
    tile_start = torch.empty(n_tiles + 2, dtype=torch.int64, device=device)
    ws = _ws((n_tiles + 1) * 8 + query("msp_scan_workspace_size", I64(n_tiles)), device)
    call("msp_tile_rulebook", ptr(m), K, n, tr, ptr(tile_start), None, None, None, 0, ptr(ws), ws.numel(), s)
    out = dict(tile_start=tile_start, tile_rows=tr)

    def fill(counts):
        n_chunks, max_chunks = counts
        chunk_off = torch.empty(max(n_chunks, 1), dtype=torch.uint8, device=device)
        chunk_src = torch.empty(max(n_chunks, 1) * CHUNK, dtype=torch.int32, device=device)
        # uint16 row-in-tile; stored in an int16 tensor (same bytes, rows < 2^15)
        chunk_row = torch.empty(max(n_chunks, 1) * CHUNK, dtype=torch.int16, device=device)
        if n_chunks:
            call("msp_tile_rulebook", ptr(m), K, n, tr, ptr(tile_start), ptr(chunk_off), ptr(chunk_src),
                 ptr(chunk_row), n_chunks, ptr(ws), ws.numel(), s)
        out.update(chunk_off=chunk_off, chunk_src=chunk_src, chunk_row=chunk_row, n_chunks=n_chunks,
                   max_chunks=max_chunks)
    _later(tile_start[n_tiles:], fill)
    return out


LOCAL_TILE_ROWS = 128


def local_rulebook(nbr, K, n, device, s, tile_rows=LOCAL_TILE_ROWS, lists_only=False):
    """msp_tile_local: count (one host read of the total, deferred in a replay), then fill (lists_only: the
    distinct-row lists without the row grouping and local indices, for the chunk-local weight gradient alone)."""
    T = int(tile_rows)
    n_tiles = (n + T - 1) // T
    u_start = torch.empty(n_tiles + 2, dtype=torch.int64, device=device)
    ws = _ws(query("msp_tile_local_workspace_size", I64(n), T), device)
    call("msp_tile_local", ptr(nbr), K, n, T, ptr(u_start), None, 0, None, None, None, ptr(ws), ws.numel(), s)
    out = dict(u_start=u_start, tile_rows=T, n_tiles=n_tiles)

    def fill(counts):
        total, max_u = counts
        u_rows = torch.empty(max(total, 1), dtype=torch.int32, device=device)
        out.update(u_rows=u_rows, total=total, max_u=max_u)
        if lists_only:
            if n_tiles:
                call("msp_tile_local", ptr(nbr), K, n, T, ptr(u_start), ptr(u_rows), max(total, 1), None, None,
                     None, ptr(ws), ws.numel(), s)
            return
        lidx = torch.empty((K, max(n_tiles * T, 1)), dtype=torch.int16, device=device)  # uint16 bits
        perm = torch.empty(max(n_tiles * T, 1), dtype=torch.int32, device=device)
        # conv_x6s's per-tile offset lists (128-row tiles, K <= 27)
        wave_off = torch.empty(max(n_tiles * 64, 1), dtype=torch.uint8, device=device) \
            if T == 128 and K <= 27 else None
        if n_tiles:
            call("msp_tile_local", ptr(nbr), K, n, T, ptr(u_start), ptr(u_rows), max(total, 1), ptr(lidx),
                 ptr(perm), ptr(wave_off) if wave_off is not None else None, ptr(ws), ws.numel(), s)
        out.update(lidx=lidx, perm=perm, wave_off=wave_off)
    if n_tiles:
        _later(u_start[n_tiles:], fill)
    else:
        fill((0, 0))
    return out


class PairLists:
    """Per-offset (in, out) pair lists of an offset-major map, plus the chunk
    and block partitions used by msp_conv_pairs / msp_conv_wgrad.

    The per-offset counts (the SCN rulebook size, the MAC counter) are taken
    when the rules are built; the lists themselves are filled on first use of
    `pair_in` / `pair_out` (recorded in the plan, so a prefetch of the next
    batch builds them ahead): at levels whose convolutions and weight gradients
    all run on the tile-local / chunk forms nothing reads them.  The fill needs
    no host read, so a first use inside a graph capture is captured; the fill reads the block offsets the
    count left in its workspace, so the workspace stays on the object (and with it in Metadata.tensors(), which
    a capturer keeps alive and a consumer stream marks) for as long as the lists may be filled."""

    def __init__(self, m, K, n, device, s, plan=None, key=None):
        nrb = max(1, (n + 2047) // 2048)
        mm = K * nrb
        ws = _ws((2 * mm + 1) * 8 + query("msp_scan_workspace_size", I64(mm)), device)
        self.off_start = torch.empty(K + 1, dtype=torch.int64, device=device)
        call("msp_pair_lists", ptr(m), K, n, None, None, 0, ptr(self.off_start), ptr(ws), ws.numel(), s)
        # the filling call reuses the count's workspace (kept: a fill captured into a graph reads it at replay)
        self._m, self._n, self._ws, self._dev = m, n, ws, device
        self._plan, self._key = plan, key
        self._pin = self._pout = None
        self.K = K
        _later(self.off_start, self._counted)

    def _counted(self, starts):
        self.total = starts[-1]
        self.counts = [starts[o + 1] - starts[o] for o in range(self.K)]
        # 16-pair chunks per offset (msp_conv_pairs): the starts computed on the device from off_start (a
        # host-to-device copy from pageable memory would wait for a copy kernel that queues beside the step)
        self.n_chunks = sum((c + CHUNK - 1) // CHUNK for c in self.counts)

    def _chunk_starts(self):
        """16-pair chunk starts per offset (msp_conv_pairs / the pair-list weight gradient), computed on the
        device from off_start (a host-to-device copy from pageable memory would wait for a copy kernel that
        queues beside the step) when the lists are filled -- five small kernels that most levels, whose
        convolutions and weight gradients take the tile-local and chunk forms, never need."""
        cs = torch.zeros(self.K + 1, dtype=torch.int64, device=self._dev)
        torch.cumsum(torch.div(self.off_start.diff() + (CHUNK - 1), CHUNK, rounding_mode="floor"), 0, out=cs[1:])
        self.chunk_start = cs
        return cs

    def __getattr__(self, name):
        # a count still queued in the replay in progress: read it now
        if name in ("total", "counts", "n_chunks", "chunk_start") and _defer() is not None:
            _defer().flush()
            if name in self.__dict__:
                return self.__dict__[name]
        if name == "chunk_start" and "total" in self.__dict__:
            return self._chunk_starts()
        raise AttributeError(name)

    def fill(self):
        if self._pin is None:
            if "total" not in self.__dict__:   # counted in a replay, not read yet: fill once it is
                _defer().then(self.fill)
                return self
            if self._plan is not None:
                self._plan.append(("pairs", self._key))
            pin = torch.empty(max(self.total, 1), dtype=torch.int32, device=self._dev)
            pout = torch.empty(max(self.total, 1), dtype=torch.int32, device=self._dev)
            if self.total:
                call("msp_pair_lists", ptr(self._m), self.K, self._n, ptr(pin), ptr(pout), self.total,
                     ptr(self.off_start), ptr(self._ws), self._ws.numel(), _lib.stream(self._dev))
            self._pin, self._pout = pin, pout
            if "chunk_start" not in self.__dict__:
                self._chunk_starts()
        return self

    @property
    def pair_in(self):
        return self.fill()._pin

    @property
    def pair_out(self):
        return self.fill()._pout


DENSE_LOG2_WINDOW = 12  # rows of one mask-sorting window of msp_dense_order


class SubmRules:
    def __init__(self, level, filter_size):
        self._plan, self._key = level.plan, ("subm", level.size, filter_size)
        dev, s = level.device, _lib.stream(level.device)
        K = filter_size ** 3
        self.K, self.filter_size = K, filter_size
        V = level.n
        table, cap = level.hash()
        self.nbr = torch.empty((K, max(V, 1)), dtype=torch.int32, device=dev)
        # the rulebook size counted as the map is written (round 5; the pair lists' count pass over the map ran
        # for every level, though most never fill the lists)
        self._nr = torch.empty(1, dtype=torch.int64, device=dev)
        ws = _ws(query("msp_subm_map_workspace_size", I64(V), filter_size), dev)
        call("msp_subm_map_counted", ptr(level.keys), V, level.log2, level.size, filter_size, ptr(table), cap,
             ptr(self.nbr), ptr(self._nr), ptr(ws), ws.numel(), s)
        self._tiles = {}
        self._locals = {}
        self._wchunk = None
        self._dense = None
        self._map, self._n = self.nbr, V
        self._pairs = None
        _later(self._nr, self._counted)

    def _counted(self, vals):
        self._n_rules = vals[0]

    @property
    def n_rules(self):
        """SCN's rulebook size (centre included); a count still queued in the replay in progress is read now."""
        if "_n_rules" not in self.__dict__ and _defer() is not None:
            _defer().flush()
        if "_n_rules" not in self.__dict__:  # a replay whose flush failed left the count unread: read it now
            self._n_rules = int(_host(self._nr)[0])
        return self._n_rules

    @property
    def pairs(self):
        """Per-offset pair lists of the map (the pair-list weight gradient), counted on first use."""
        if self._pairs is None:
            self._pairs = PairLists(self.nbr, self.K, self._n, self.nbr.device, _lib.stream(self.nbr.device),
                                    self._plan, self._key)
        return self._pairs

    def dense_order(self):
        """(perm, permuted neighbour map) for the dense row-group convolution
        (msp_dense_order: rows sorted by neighbour mask inside 4096-row
        windows), built on first use; (None, nbr) when K > 32."""
        if self._dense is None:
            self._plan.append(("dense", self._key))
            V, K = self._n, self.K
            if K > 32 or V == 0:
                self._dense = (None, self.nbr)
            else:
                dev, s = self.nbr.device, _lib.stream(self.nbr.device)
                perm = torch.empty(V, dtype=torch.int32, device=dev)
                nbr_p = torch.empty((K, V), dtype=torch.int32, device=dev)
                wsb = int(_lib.query("msp_dense_order_workspace_size", _lib.I64(V), K, DENSE_LOG2_WINDOW))
                ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
                call("msp_dense_order", ptr(self.nbr), K, V, DENSE_LOG2_WINDOW, ptr(perm), ptr(nbr_p), ptr(ws), wsb,
                     s)
                self._dense = (perm, nbr_p)
        return self._dense

    def local(self, tile_rows=LOCAL_TILE_ROWS):
        """Tile-local rulebook (msp_tile_local) for msp_conv_local, built on first use: per tile the sorted
        distinct input rows, the rows' order inside the tile and the local index of every neighbour."""
        t = self._locals.get(tile_rows)
        if t is None:
            self._plan.append(("local", self._key, tile_rows))
            t = self._locals[tile_rows] = local_rulebook(self.nbr, self.K, self._n, self.nbr.device,
                                                         _lib.stream(self.nbr.device), tile_rows)
        return t

    def lists(self, tile_rows=LOCAL_TILE_ROWS):
        """Each tile's sorted distinct input rows (the tile-local rulebook's u_start / u_rows): the full
        rulebook's when a tile-local convolution built it, else a lists-only build (no row grouping)."""
        t = self._locals.get(tile_rows)
        if t is None:
            t = self.__dict__.setdefault("_lists", {}).get(tile_rows)
        if t is None:
            self._plan.append(("lists", self._key, tile_rows))
            t = self._lists[tile_rows] = local_rulebook(self._map, self.K, self._n, self._map.device,
                                                        _lib.stream(self._map.device), tile_rows, lists_only=True)
        return t

    def wgrad_index(self, wait=False):
        """msp_wgrad_chunk_index over the 128-row tile rulebook and the tile-local lists of each tile's distinct
        input rows for msp_conv_wgrad_chunk, built on first use.  Rules whose input row lies past the rows a tile
        stages (a tile listing more than msp_wgrad_chunk_cap rows) are listed apart (msp_wgrad_far_list, sorted)
        and added by msp_conv_wgrad_far: the chunk form serves every map.

        Inside a replay whose counts are not read yet this returns the _PENDING sentinel (the index is built when
        the replay flushes its reads); wait=True (every consumer of the index) flushes them first, so the caller
        always gets the index itself."""
        if self._wchunk is _PENDING or (isinstance(self._wchunk, dict) and "chunk_lr" not in self._wchunk):
            if not wait:
                return self._wchunk
            d = _defer()
            if d is not None:
                d.flush()
            # the replay ended without deciding or without filling the index (its flush failed): build it now
            w = self._wchunk
            if w is _PENDING or (isinstance(w, dict) and "chunk_lr" not in w):
                self._wchunk = None
        if self._wchunk is None and LOCAL_CHUNK_INDEX:
            full = self._locals.get(128)
            if full is not None and "lidx" not in full:  # a replay's counts not read yet: decide once they are
                self._wchunk = _PENDING

                def decide_full():
                    self._wchunk = None
                    self.wgrad_index()
                _defer().then(decide_full)
                return self._wchunk
            if full is not None and full["max_u"] <= int(query("msp_wgrad_chunk_cap")):
                self._plan.append(("wchunk", self._key))
                self._wchunk = self._local_chunk_index(full)
                return self._wchunk
        if self._wchunk is None:
            loc = self.lists()
            tiles = self.tiles_for(128)
            if "max_u" not in loc or "n_chunks" not in tiles:
                # in a replay, counts not read yet: build the index once they are read (one read for both)
                self._wchunk = _PENDING

                def decide():
                    self._wchunk = None
                    self.wgrad_index()
                _defer().then(decide)
                return self._wchunk
            self._plan.append(("wchunk", self._key))
            dev, s = self._map.device, _lib.stream(self._map.device)
            lr = torch.empty(max(tiles["n_chunks"], 1) * CHUNK, dtype=torch.int32, device=dev)
            over = loc["max_u"] > int(query("msp_wgrad_chunk_cap"))
            n_far = torch.zeros(1, dtype=torch.int64, device=dev) if over else None
            if self._n:
                call("msp_wgrad_chunk_index", ptr(tiles["tile_start"]), ptr(tiles["chunk_src"]),
                     ptr(tiles["chunk_row"]), I64(self._n), ptr(loc["u_start"]), ptr(loc["u_rows"]), ptr(lr),
                     ptr(n_far), s)
            idx = self._wchunk = dict(tiles=tiles, chunk_lr=lr, u_start=loc["u_start"], u_rows=loc["u_rows"],
                                      n_far=0)
            if over and self._n:
                def far(vals):
                    nf = vals[0]
                    idx["n_far"] = nf
                    if nf:
                        key = torch.empty(nf, dtype=torch.int64, device=dev)
                        tile = torch.empty(nf, dtype=torch.int32, device=dev)
                        ws = _ws(query("msp_wgrad_far_workspace_size", I64(nf)), dev)
                        call("msp_wgrad_far_list", ptr(tiles["tile_start"]), ptr(tiles["chunk_off"]), ptr(lr),
                             I64(self._n), I64(nf), ptr(key), ptr(tile), ptr(ws), ws.numel(), _lib.stream(dev))
                        idx.update(far_key=key, far_tile=tile, far_ws=ws)
                _later(n_far, far)
        return self._wchunk

    def _local_chunk_index(self, loc):
        """The chunk weight gradient's index from the full tile-local rulebook (msp_local_chunk_index: count, one
        host read of the chunk total -- deferred in a replay -- then fill): no 128-row tile rulebook and no
        binary searches where a tile-local convolution built that rulebook anyway."""
        dev, s, n = self._map.device, _lib.stream(self._map.device), self._n
        n_tiles = (n + 127) // 128
        tile_start = torch.empty(n_tiles + 2, dtype=torch.int64, device=dev)
        ws = _ws(query("msp_tile_local_workspace_size", I64(n), 128), dev)
        call("msp_local_chunk_index", ptr(loc["lidx"]), ptr(loc["perm"]), self.K, n, ptr(tile_start), None, None,
             0, ptr(ws), ws.numel(), s)
        tiles = dict(tile_start=tile_start, tile_rows=128)
        idx = dict(tiles=tiles, u_start=loc["u_start"], u_rows=loc["u_rows"], n_far=0, ws=ws)

        def fill(counts):
            n_chunks, max_chunks = counts
            chunk_off = torch.empty(max(n_chunks, 1), dtype=torch.uint8, device=dev)
            lr = torch.empty(max(n_chunks, 1) * CHUNK, dtype=torch.int32, device=dev)
            if n_chunks:
                call("msp_local_chunk_index", ptr(loc["lidx"]), ptr(loc["perm"]), self.K, n, ptr(tile_start),
                     ptr(chunk_off), ptr(lr), n_chunks, ptr(ws), ws.numel(), s)
            tiles.update(chunk_off=chunk_off, n_chunks=n_chunks, max_chunks=max_chunks)
            idx["chunk_lr"] = lr
        if n_tiles:
            _later(tile_start[n_tiles:], fill)
        else:
            fill((0, 0))
        return idx

    def note_use(self, purpose, c_in, c_out):
        """Record in the plan that a convolution / weight gradient with these channel counts runs over these
        rules: a replay then builds what that call selects for ITS batch's sizes (ops.prepare)."""
        e = ("use", self._key, purpose, int(c_in), int(c_out))
        seen = self.__dict__.setdefault("_uses", set())
        if e not in seen:
            seen.add(e)
            self._plan.append(e)

    def tiles_for(self, tile_rows):
        """Tile rulebook with tile_rows-row tiles, built on first use."""
        t = self._tiles.get(tile_rows)
        if t is None:
            self._plan.append(("tiles", self._key, tile_rows))
            t = self._tiles[tile_rows] = tile_rulebook(self._map, self.K, self._n, self._map.device,
                                                       _lib.stream(self._map.device), tile_rows)
        return t


class DownRules:
    """Strided (size == stride) relation between a fine and a coarse level."""

    def __init__(self, fine, coarse, parent_of, child_start, log2_stride):
        self._plan, self._key = fine.plan, ("down", fine.size, 1 << log2_stride)
        dev, s = fine.device, _lib.stream(fine.device)
        K = 8 ** log2_stride
        self.K = K
        self.parent_of = parent_of
        self.child_start = child_start
        self.down = torch.empty((K, max(coarse.n, 1)), dtype=torch.int32, device=dev)
        call("msp_down_map", ptr(fine.keys), fine.n, ptr(parent_of), fine.log2, log2_stride, ptr(self.down),
             coarse.n, s)
        self._tiles = {}
        self._map, self._n = self.down, coarse.n
        # pair_in = fine row, pair_out = coarse row, grouped by child offset
        self.pairs = PairLists(self.down, K, coarse.n, dev, s, self._plan, self._key)
        # the chunk weight gradient over the child map (round 6): 128-coarse-row tiles, each tile's distinct fine
        # rows staged (ops.ConvolutionFunction / DeconvolutionFunction backward)
        self._locals = {}
        self._wchunk = None

    tiles_for = SubmRules.tiles_for
    note_use = SubmRules.note_use
    lists = SubmRules.lists
    wgrad_index = SubmRules.wgrad_index
    _local_chunk_index = SubmRules._local_chunk_index


class Level:
    def __init__(self, size, log2, keys, n, device, plan=None):
        self.size, self.log2, self.keys, self.n, self.device = int(size), int(log2), keys, int(n), device
        self.plan = plan if plan is not None else []
        self._hash = None
        self.subm = {}
        self.down = {}  # stride -> (coarse size, DownRules)

    def hash(self):
        if self._hash is None:
            cap = int(query("msp_hash_capacity", I64(self.n)))
            table = torch.empty((2 * cap,), dtype=torch.int64, device=self.device)  # {key, value} slots
            call("msp_hash_build", ptr(self.keys), self.n, ptr(table), cap, _lib.stream(self.device))  # (empties it)
            self._hash = (table, cap)
        return self._hash

    def subm_rules(self, filter_size):
        r = self.subm.get(filter_size)
        if r is None:
            self.plan.append(("subm", self.size, filter_size))
            r = self.subm[filter_size] = SubmRules(self, filter_size)
        return r


class InputRules:
    """Point <-> voxel relation of InputLayer/OutputLayer."""

    def __init__(self, n_points, perm, p2v, vstart, batch_size):
        self.n_points, self.perm, self.p2v, self.vstart, self.batch_size = n_points, perm, p2v, vstart, batch_size
        self.batch_monotonic = False  # batch column non-decreasing along the points
        self.scene_starts = None      # host list: first point of batch id b, b = 0..batch_size (monotonic only)

    def scene_ranges_match(self, batch_offsets):
        """True when scene b of `batch_offsets` (dataset/data.py:142,209) is exactly the points of batch id b
        (decided on the host from the counts read back with the voxel count; no device read)."""
        off = [int(o) for o in batch_offsets]
        B = len(off) - 1
        if B < 1 or not self.batch_monotonic or self.scene_starts is None or self.batch_size > B:
            return False
        st = self.scene_starts + [self.n_points] * (B + 1 - len(self.scene_starts))
        return st[:B + 1] == off


class Metadata:
    def __init__(self, device):
        self.device = torch.device(device)
        self.levels = {}
        self.input = None
        # every lazily built rulebook, in build order: a later Metadata of the
        # same network can build them all up front (replay, prefetch)
        self.plan = []

    # ------------------------------------------------------------ level 0
    def build_input(self, coords, spatial_size):
        dev = self.device
        s = _lib.stream(dev)
        size = int(spatial_size)
        log2 = _log2_ceil(size)
        coords = coords.to(dev, torch.int64).contiguous()
        if coords.dim() != 2 or coords.size(1) != 4:
            raise ValueError(f"InputLayer expects coords (N, 4) [x, y, z, batch], got {tuple(coords.shape)}")
        n = coords.size(0)
        keys = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        vals = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        stats = torch.zeros(3, dtype=torch.int64, device=dev)
        if n:
            call("msp_point_keys", ptr(coords), n, 4, log2, size, ptr(keys), ptr(vals), ptr(stats), s)
        n_bad, max_b, n_desc = _host(stats)
        if n_bad:
            raise ValueError(f"InputLayer: {n_bad} points outside [0, {size})^3 or with a negative batch index")
        end_bit = min(64, 3 * log2 + max(1, int(max_b).bit_length()))
        if 3 * log2 + int(max_b).bit_length() > 63:
            raise ValueError("InputLayer: batch index too large for 64-bit keys")
        skeys = torch.empty_like(keys)
        perm = torch.empty_like(vals)
        if n:
            wsb = int(query("msp_sort_workspace_size", I64(n), end_bit))
            ws = _ws(wsb, dev)
            call("msp_sort_pairs", ptr(keys), ptr(skeys), ptr(vals), ptr(perm), n, end_bit, ptr(ws), ws.numel(), s)
        seg_of = torch.empty_like(vals)
        p2v = torch.empty_like(vals)
        uniq = torch.empty_like(keys)
        vstart = torch.empty(n + 1, dtype=torch.int32, device=dev)
        n_batch = int(max_b) + 1 if n else 0
        monotonic = n_desc == 0
        # one read-back: [voxel count, scene starts of a non-decreasing batch column (msp_batch_starts)]
        tail = torch.empty(2 + (n_batch if monotonic else 0), dtype=torch.int64, device=dev)  # (all read are written)
        ws = _ws(((n + 2047) // 2048 + 1) * 8, dev)
        call("msp_segment", ptr(skeys), n, 0, ptr(perm), ptr(seg_of), ptr(p2v), ptr(uniq), ptr(vstart), ptr(tail),
             ptr(ws), ws.numel(), s)
        if monotonic:
            call("msp_batch_starts", ptr(coords), n, 4, n_batch, ptr(tail[1:]), s)
        got = _host(tail)
        V = int(got[0])
        lvl = Level(size, log2, uniq[:max(V, 1)], V, dev, self.plan)
        self.levels[size] = lvl
        self.input = InputRules(n, perm[:n], p2v[:n], vstart[:V + 1], n_batch)
        self.input.batch_monotonic = monotonic
        self.input.scene_starts = [int(v) for v in got[1:]] if monotonic else None
        return lvl

    def level(self, size):
        lvl = self.levels.get(int(size))
        if lvl is None:
            raise RuntimeError(f"no active sites at spatial size {size} in this metadata")
        return lvl

    # ------------------------------------------------------------ coarsening
    def downsample(self, size, stride):
        """Return (coarse Level, DownRules) for a size==stride convolution or
        pooling from spatial size `size`."""
        fine = self.level(size)
        stride = int(stride)
        if stride & (stride - 1) or stride not in (2, 4):
            raise NotImplementedError(f"strided ops support filter_size == stride in {{2, 4}}, got {stride}")
        if fine.size % stride:
            raise ValueError(f"spatial size {fine.size} is not divisible by stride {stride}")
        hit = fine.down.get(stride)
        if hit is not None:
            return self.levels[hit[0]], hit[1]
        self.plan.append(("down", fine.size, stride))
        k = stride.bit_length() - 1
        if fine.log2 < k:
            raise ValueError("spatial size too small for this stride")
        dev = self.device
        s = _lib.stream(dev)
        n = fine.n
        parent = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        uniq = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        cstart = torch.empty(n + 1, dtype=torch.int32, device=dev)
        nu = torch.empty(1, dtype=torch.int64, device=dev)  # (msp_segment writes it)
        ws = _ws(((n + 2047) // 2048 + 1) * 8, dev)
        call("msp_segment", ptr(fine.keys), n, 3 * k, None, ptr(parent), None, ptr(uniq), ptr(cstart), ptr(nu),
             ptr(ws), ws.numel(), s)
        got = []
        _later(nu, got.extend)
        _resolve()   # in a replay: one read for Vc and every count queued since the last one
        Vc = got[0]
        csize = fine.size // stride
        coarse = self.levels.get(csize)
        if coarse is None:
            coarse = Level(csize, fine.log2 - k, uniq[:max(Vc, 1)], Vc, dev, self.plan)
            self.levels[csize] = coarse
        elif coarse.n != Vc:
            raise RuntimeError("inconsistent coarse level")
        rules = DownRules(fine, coarse, parent[:max(n, 1)], cstart[:Vc + 1], k)
        fine.down[stride] = (csize, rules)
        return coarse, rules

    def upsample_rules(self, coarse_size, stride):
        """DownRules linking the existing fine level (coarse_size*stride) to
        `coarse_size` (Deconvolution / UnPooling)."""
        fine_size = int(coarse_size) * int(stride)
        fine = self.levels.get(fine_size)
        if fine is None or int(stride) not in fine.down:
            raise RuntimeError(f"no strided relation {fine_size} -> {coarse_size}: a Deconvolution/UnPooling needs "
                               "the matching Convolution/MaxPooling earlier in the same forward")
        return fine, fine.down[int(stride)][1]

    # ------------------------------------------------------------ replay / prefetch
    def _rules(self, key):
        kind, size, param = key
        if kind == "subm":
            return self.level(size).subm_rules(param)
        return self.downsample(size, param)[1]

    def replay(self, plan):
        """Build, in order, the rulebooks another forward of the same network
        requested (its `plan`); later requests then find them built (their count reads batched:
        _Deferred).  Rules with recorded uses ("use": a convolution or weight gradient and its
        channel counts) get what those uses select for this batch's sizes
        (ops.prepare) instead of the concrete rulebooks the other batch built."""
        if not DEFER_READS:
            return self._replay(plan)
        outer = _defer()
        _TLS.defer = _Deferred(torch.cuda.current_stream(self.device))
        try:
            self._replay(plan)
            _TLS.defer.flush()
        finally:
            _TLS.defer = outer
            # a flush that raised leaves weight-gradient indices undecided or half-built (no chunk words yet):
            # forget them (built again on use); the rulebook sizes are read on use (SubmRules.n_rules)
            for lvl in self.levels.values():
                for r in getattr(lvl, "subm", {}).values():
                    w = getattr(r, "_wchunk", None)
                    if w is _PENDING or (isinstance(w, dict) and "chunk_lr" not in w):
                        r._wchunk = None

    def _replay(self, plan):
        from . import ops
        used = {e[1] for e in plan if e[0] == "use"}
        for entry in plan:
            # what the recorded uses select is rebuilt by ops.prepare; pair lists too (the weight gradient falls
            # back to them only when its chunk form does not fit, the strided consumers record a "pairs" use)
            if entry[0] in ("tiles", "dense", "local", "lists", "wchunk", "pairs") and entry[1] in used:
                continue
            if entry[0] == "use":
                rules = self._rules(entry[1])
                rules.note_use(entry[2], entry[3], entry[4])
                ops.prepare(rules, entry[2], entry[3], entry[4])
            elif entry[0] == "down":
                self.downsample(entry[1], entry[2])
            elif entry[0] == "subm":
                self.level(entry[1]).subm_rules(entry[2])
            elif entry[0] == "tiles":
                self._rules(entry[1]).tiles_for(entry[2])
            elif entry[0] == "dense":
                self._rules(entry[1]).dense_order()
            elif entry[0] == "local":
                self._rules(entry[1]).local(entry[2])
            elif entry[0] == "lists":
                self._rules(entry[1]).lists(entry[2])
            elif entry[0] == "wchunk":
                self._rules(entry[1]).wgrad_index()
            elif entry[0] == "pairs":
                self._rules(entry[1]).pairs.fill()

    def tensors(self):
        """Every device tensor this metadata holds (for stream bookkeeping)."""
        out, seen = [], set()

        def walk(v):
            if torch.is_tensor(v):
                out.append(v)
            elif isinstance(v, dict):
                for x in v.values():
                    walk(x)
            elif isinstance(v, (list, tuple)):
                for x in v:
                    walk(x)
            elif isinstance(v, (Level, SubmRules, DownRules, PairLists, InputRules)) and id(v) not in seen:
                seen.add(id(v))
                for k, x in vars(v).items():
                    if k not in ("_plan", "plan", "_m"):
                        walk(x)
        walk(self.levels)
        walk(self.input)
        return out

    def locations(self, size):
        lvl = self.level(size)
        out = torch.empty((max(lvl.n, 1), 4), dtype=torch.int64, device=self.device)
        if lvl.n:
            call("msp_decode_keys", ptr(lvl.keys), lvl.n, lvl.log2, ptr(out), _lib.stream(self.device))
        return out[:lvl.n]


# ---------------------------------------------------------------- prefetch
# Input pipelining: the metadata of the NEXT batch (voxelisation, every
# rulebook the network requested last time) is built on a side stream while
# the current step's backward still runs on the compute stream; the next
# InputLayer forward then finds it ready (its stream waits on an event) and
# the forward issues no device-to-host reads at all.  Nothing is skipped:
# each batch's metadata is still built once, inside the step before it.
# device index -> [(coords tensor, its key, Metadata, event), ...]: at most PREFETCH_DEPTH pending entries per
# device (a newer prefetch drops the oldest beyond that); an entry holds the coords tensor itself and a hit needs
# the very same tensor object (not just the same address), so freed coords whose memory was handed to a new tensor
# can never pick up another batch's rulebooks.
_PREFETCHED = {}
_SIDE = {}
_CAPTURED = []
_LOCK = threading.Lock()  # _PREFETCHED / _CAPTURED: a prefetch may run on a worker thread beside a capture
# Pending entries kept per device: 1 (the default) -- the next batch; 2 -- a worker thread prefetches the batch
# after next while the next one's step is captured (bench.py --prefetch-thread).
PREFETCH_DEPTH = 1
BUILD_EVENT_TIMING = False  # True: the build events carry timestamps (bench.py BENCH_HOST_TIMING diagnostics)
PREFETCH_PRIORITY = 0


def _coords_key(coords, spatial_size):
    return (coords.data_ptr(), tuple(coords.shape), coords.dtype, coords._version, int(spatial_size))


def prefetch(coords, spatial_size, plan, wait_for_producer=True):
    """Build Metadata for `coords` (device, (N, 4) int64) on a side stream.
    wait_for_producer: order the side stream after all work already queued on
    the current stream (safe for coords made by queued kernels); False when
    coords have long been complete on the device (more overlap)."""
    dev = coords.device
    if dev.type != "cuda":
        raise RuntimeError("sparseconvnet.prefetch: coords must be on a HIP device")
    with _LOCK:
        pend = _PREFETCHED.setdefault(dev.index, [])
        # an unconsumed entry for the same coords, and the oldest beyond the depth, are dropped (memory goes back)
        pend[:] = [e for e in pend if e[0] is not coords][-(PREFETCH_DEPTH - 1):] if PREFETCH_DEPTH > 1 else []
        # one side stream per (device, priority): a later change of PREFETCH_PRIORITY takes effect
        side = _SIDE.get((dev.index, PREFETCH_PRIORITY))
        if side is None:
            side = _SIDE[(dev.index, PREFETCH_PRIORITY)] = torch.cuda.Stream(dev, priority=PREFETCH_PRIORITY)
    cur = torch.cuda.current_stream(dev)
    if isinstance(wait_for_producer, torch.cuda.Event):
        side.wait_event(wait_for_producer)
    elif wait_for_producer:
        side.wait_stream(cur)
    with torch.cuda.stream(side):
        m = Metadata(dev)
        m.build_input(coords, spatial_size)
        m.replay(plan)
        ev = torch.cuda.Event(enable_timing=BUILD_EVENT_TIMING)
        ev.record(side)
    with _LOCK:
        pend = _PREFETCHED.setdefault(dev.index, [])
        pend[:] = [e for e in pend if e[0] is not coords][-(PREFETCH_DEPTH - 1):] if PREFETCH_DEPTH > 1 else []
        pend.append((coords, _coords_key(coords, spatial_size), m, ev))
    return m


def take_prefetched(coords, spatial_size):
    """The Metadata prefetched for this very coords tensor (popped), with the
    current stream ordered after its build and its tensors marked as used by
    the current stream; None if there is none."""
    if not _PREFETCHED:
        return None
    with _LOCK:
        pend = _PREFETCHED.get(coords.device.index) or []
        hit = next((e for e in pend if e[0] is coords), None)
        if hit is None or hit[1] != _coords_key(coords, spatial_size):
            return None
        pend[:] = [e for e in pend if e is not hit]   # by identity (== on the tuples would compare tensors)
    _, _, m, ev = hit
    cur = torch.cuda.current_stream(coords.device)
    if torch.cuda.is_current_stream_capturing():
        # inside a graph capture (bench.py --graph): the replaying stream waits on the build before the graph
        # runs (prefetch_event, taken before the capture), and the Metadata must outlive every replay: it is
        # parked here until the capturer takes it with captured_metadata()
        with _LOCK:
            _CAPTURED.append(m)
        return m
    cur.wait_event(ev)
    for t in m.tensors():
        t.record_stream(cur)
    return m


def pending_count():
    """Prefetched entries not consumed yet, over all devices."""
    with _LOCK:
        return sum(len(v) for v in _PREFETCHED.values())


def captured_metadata():
    """The Metadata consumed inside graph captures since the last call (the capturer keeps them alive for
    as long as it replays the graph)."""
    with _LOCK:
        out = list(_CAPTURED)
        _CAPTURED.clear()
    return out


def prefetch_event(device, coords=None):
    """The build event of the entry pending on `device` for `coords` (None: the newest entry; None if there is
    none): a stream that will replay a graph capturing the consumption of that entry must wait on it first."""
    with _LOCK:
        pend = _PREFETCHED.get(torch.device(device).index) or []
        if coords is not None:
            pend = [e for e in pend if e[0] is coords]
        return pend[-1][3] if pend else None
