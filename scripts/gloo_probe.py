"""Where the two-rank shared-device rehearsal's wall time goes (bench.py BENCH_BACKEND=gloo BENCH_SHARE_DEVICE=1):
times one gloo all_reduce of the headline UNet's flat gradient buffer (30.1 M fp32 = 120 MB) between two ranks on
cuda:0, for a device tensor (gloo stages it through host memory) and a host tensor, with torch's default intra-op
thread count and with it bounded to the process's CPU share / world.

Usage: python scripts/gloo_probe.py   (starts its two ranks itself; env N_FLOATS, REPS)"""
import os
import socket
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def _cores():
    from bench import host_cores
    return host_cores()[0]


def run(rank, world, port, n, reps):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    default_threads = torch.get_num_threads()
    for threads in (default_threads, max(1, _cores() // world)):
        torch.set_num_threads(threads)
        for where in (["cuda:0"] if torch.cuda.device_count() else []) + ["cpu"]:
            t = torch.ones(n, dtype=torch.float32, device=where)
            dist.all_reduce(t)  # warm-up
            if where != "cpu":
                torch.cuda.synchronize()
            dist.barrier()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                dist.all_reduce(t)
                if where != "cpu":
                    torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            if rank == 0:
                print(f"gloo all_reduce {n * 4 / 1e6:.0f} MB on {where:6s} torch threads {threads:4d}: "
                      f"median {1e3 * ts[len(ts) // 2]:8.1f} ms  min {1e3 * ts[0]:8.1f} ms  "
                      f"({n * 4 / ts[len(ts) // 2] / 1e9:.2f} GB/s)", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    n = int(os.environ.get("N_FLOATS", 30104372))
    reps = int(os.environ.get("REPS", 5))
    print(f"host cores (affinity, cgroup quota): {_cores()}; torch default threads {torch.get_num_threads()}",
          flush=True)
    mp.spawn(run, args=(2, port, n, reps), nprocs=2)
