"""NetworkInNetwork GEMM shapes of the headline UNet on msp_nin_gemm (split-bf16 MFMA) (x[V, 2a] @ W[2a, a] and
the backward-data g[V, a] @ W^T) on hipBLASLt vs rocBLAS (torch's
preferred_blas_library), HIP-event timed; HBM roofline = (V*(cin+cout))*4 B / 8 TB/s."""
import torch
dev = "cuda:0"
shapes = [(1349716, 64, 32), (565253, 128, 64), (149654, 192, 96), (36553, 256, 128)]
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g_; g_.add_path()
from sparseconvnet import ops, _lib
for lib in ("msp", "cublaslt", "cublas"):
    if lib != "msp":
        torch.backends.cuda.preferred_blas_library(lib)
    for V, ci, co in shapes:
        x = torch.randn(V, ci, device=dev); w = torch.randn(ci, co, device=dev)
        g = torch.randn(V, co, device=dev)
        wt = w.t().contiguous()
        mm = (lambda a, b: ops.nin_gemm(a, b)) if lib == "msp" else (lambda a, b: a @ b)
        for name, fn in (("fwd", lambda: mm(x, w)), ("bwd", lambda: mm(g, wt))):
            for _ in range(3): fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20): fn()
            e.record(); torch.cuda.synchronize()
            us = s.elapsed_time(e) / 20 * 1e3
            roof = V * (ci + co) * 4 / 8e12 * 1e6
            print(f"{lib:9s} {name} V={V:8d} {ci:3d}->{co:3d}: {us:7.1f} us  (HBM floor {roof:5.1f} us)", flush=True)
