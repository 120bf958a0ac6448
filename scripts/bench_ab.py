"""A/B of conv-path variants inside the real training step: runs bench.main()
once per variant in one process (same box, same batches), prints ms/step.
Variants (comma list in AB): tile (no dense row groups), nbr0 (dense groups in
key order), nbr (production: mask-sorted order), g<N> (dense kernel variant N,
msp_debug_conv_nbr_variant), fuse / nofuse (residual fork/join fusions on / off),
fused / foreach (Adam implementation), cw (weight gradients on a side stream), nolocal (gather forms instead of
the tile-local convolution), x6s / x6l / x6l64 (tile-local kernel forms), norec (no HIP-event recording), l0 (tile-local convolution at 32 channels too: level 0 of m = 32).  Usage: AB=tile,nbr python scripts/bench_ab.py"""
import io, json, os, sys, contextlib
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g_; g_.add_path()
import bench
from sparseconvnet import _lib, metadata, modules, ops
lib = _lib.load()
lib.msp_debug_conv_local_abl.argtypes = [__import__("ctypes").c_int]
orig_query, orig_order = _lib.query, metadata.SubmRules.dense_order
res = []
for v in os.environ.get("AB", "tile,nbr").split(","):
    _lib.query, metadata.SubmRules.dense_order = orig_query, orig_order
    lib.msp_debug_conv_nbr_variant(0)
    modules.FUSE_RESIDUAL = v != "nofuse"
    ops.CONV_LOCAL = v != "nolocal"
    lib.msp_debug_conv_local_abl({"x6s": -1, "x6l": -2, "x6l64": -4}.get(v, -3))
    lib.msp_debug_conv_local_min_ch(32 if v == "l0" else 64)
    if v == "tile":
        _lib.query = lambda name, *a: 0 if name == "msp_conv_nbr_preferred" else orig_query(name, *a)
    elif v == "nbr0":
        metadata.SubmRules.dense_order = lambda self: (None, self.nbr)
    elif v.startswith("g"):
        lib.msp_debug_conv_nbr_variant(int(v[1:]))
    sys.argv = ["bench.py", "--steps", os.environ.get("STEPS", "10"), "--warmup", "2", "--no-cpu"] + \
        (["--foreach-adam"] if v == "foreach" else []) + (["--concurrent-wgrad"] if v == "cw" else []) + (["--record", "none"] if v == "norec" else []) + (["--record", "conv"] if v == "recconv" else []) + (["--prefetch-at", "fwd"] if v == "pfwd" else []) + (["--no-prefetch"] if v == "nopf" else [])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main()
    line = [l for l in buf.getvalue().splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    res.append((v, d["ms_per_step"]))
    conv = d.get("roofline", {}).get("achieved", float("nan"))
    print(f"{v:8s} {d['ms_per_step']:.2f} ms/step  conv TF/s {conv:.1f}  {d['config']['input_pipeline'][-40:]}", flush=True)
