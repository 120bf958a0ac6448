"""Does a device-to-host copy through Tensor.cpu() let go of the GIL while it waits?  A worker thread queues
~50 ms of GPU work and reads one value back; the main thread counts Python loop iterations meanwhile."""
import threading
import time

import torch

x = torch.randn(8192, 8192, device="cuda")
torch.cuda.synchronize()


def work(read):
    y = x
    for _ in range(20):
        y = y @ x
        y = y / y.norm()
    t = time.perf_counter()
    v = read(y.sum())
    return time.perf_counter() - t, v


for name, read in (("cpu().tolist()", lambda t: t.cpu().tolist()), ("tolist()", lambda t: t.tolist()),
                   ("item()", lambda t: t.item())):
    work(read)
    out = {}
    th = threading.Thread(target=lambda: out.setdefault("r", work(read)))
    n = 0
    th.start()
    t0 = time.perf_counter()
    while th.is_alive():
        n += 1
    dt = time.perf_counter() - t0
    print(f"{name:16s} worker wait {1e3 * out['r'][0]:6.1f} ms; main thread {n} iterations in {1e3 * dt:6.1f} ms "
          f"({n / max(dt, 1e-9) / 1e6:.1f} M/s)", flush=True)
