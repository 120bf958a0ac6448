"""The training loop's optimizer on the library: torch.optim.Adam (train.py:39, ``optim.Adam(model.parameters(),
lr=1e-3)``) as one launch per step over every parameter tensor (``msp_adam_step``, csrc/msp_optim.hip).

torch's fused multi-tensor Adam takes 12 launches of ~50 us per step for the headline UNet's 203 tensors (30.1 M
floats); this is one grid over all of them (plus a one-thread step-count bump), HBM-bound on the 840 MB a step must
move.  Same update rule per element as torch's fused Adam (amsgrad off), checked against ``torch.optim.Adam`` in
tests/test_gpu_optim.py.  Graph-capturable: the step count lives on the device and the gradient pointers of the
step being captured travel in the kernel arguments."""
import ctypes

import torch

from sparseconvnet import _lib
from sparseconvnet._lib import call, ptr


class _Tensor(ctypes.Structure):  # msp_adam_tensor
    _fields_ = [("param", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p), ("exp_avg_sq", ctypes.c_void_p),
                ("n", ctypes.c_int64)]


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam's update (lr, betas, eps, weight_decay; amsgrad and maximize off) on fp32 device
    parameters, every parameter group stepping together (one device step count per optimizer).  State per
    parameter: ``exp_avg`` and ``exp_avg_sq`` as in torch (``state_dict`` layout compatible apart from the shared
    step count, kept in ``self.step_count``)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._built = None
        self._key = None
        self.step_count = None

    def _build(self):
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("wsss3d.optim.Adam: take one step eagerly before capturing steps in a graph (the first "
                               "step allocates the moments and uploads the tensor table)")
        params = [p for g in self.param_groups for p in g["params"]]
        if not params:
            self._built, self._key = [], ()
            return
        dev = params[0].device
        for p in params:
            if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.device == dev):
                raise RuntimeError("wsss3d.optim.Adam: parameters must be contiguous fp32 tensors on one HIP device")
            st = self.state[p]
            if "exp_avg" not in st:
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
        if self.step_count is None:
            self.step_count = torch.zeros(1, dtype=torch.float32, device=dev)
        # one table per group of <= MSP_ADAM_MAX_TENSORS tensors, each with its hyper-parameters
        built = []
        for g in self.param_groups:
            ps = list(g["params"])
            for k in range(0, len(ps), 256):
                part = ps[k:k + 256]
                tab = (_Tensor * len(part))()
                starts = [0]
                for i, p in enumerate(part):
                    st = self.state[p]
                    tab[i] = _Tensor(p.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), p.numel())
                    starts.append(starts[-1] + int(_lib.query("msp_adam_chunks", _lib.I64(p.numel()))))
                dtab = torch.frombuffer(bytearray(tab), dtype=torch.uint8).to(dev)
                dstart = torch.tensor(starts, dtype=torch.int64, device=dev)
                built.append((g, part, dtab, dstart, starts[-1]))
        self._built = built
        # what the table points at: a parameter moved or re-allocated (model.to(...), load_state_dict into new
        # storage, a group added) means a rebuild, never a write through a stale pointer
        self._key = self._table_key()

    def _table_key(self):
        return tuple((id(p), p.data_ptr(), self.state[p]["exp_avg"].data_ptr(), self.state[p]["exp_avg_sq"].data_ptr())
                     if p in self.state and "exp_avg" in self.state[p] else (id(p), p.data_ptr(), 0, 0)
                     for g in self.param_groups for p in g["params"])

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._built is None or self._table_key() != self._key:
            self._build()
        stream = _lib.stream(self.step_count.device) if self.step_count is not None else None
        first = True
        for g, part, dtab, dstart, n_chunks in self._built:
            grads = []
            for p in part:
                gr = p.grad
                if gr is not None:
                    if gr.dtype != torch.float32 or gr.shape != p.shape:
                        raise RuntimeError("wsss3d.optim.Adam: gradient dtype / shape does not match its parameter")
                    if not gr.is_contiguous():
                        gr = p.grad = gr.contiguous()
                grads.append(gr)
            arr = (ctypes.c_void_p * len(part))(*[ptr(gr) if gr is not None else None for gr in grads])
            b1, b2 = g["betas"]
            call("msp_adam_step", ptr(dtab), ptr(dstart), ctypes.cast(arr, ctypes.c_void_p), len(part), n_chunks,
                 ptr(self.step_count), int(first), float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                 float(g["weight_decay"]), stream)
            first = False
        return loss
