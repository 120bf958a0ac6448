# The N-rank graph path on a one-GPU box: bench.py with a one-rank RCCL group (and a gloo one) against the plain
# one-rank run -- the eager gradient all-reduce between per-step captures, as the driver's multi-GPU runs do
set -o pipefail
for v in "BENCH_DP_SELFTEST=1" "BENCH_DP_SELFTEST=gloo" "BENCH_HOST_TIMING=1"; do
  env $v BENCH_HOST_TIMING=1 timeout -k 10 300 python bench.py --no-cpu --steps 12 --family-steps 1 > gpurun_out/dpdiag.log 2>&1 || exit 1
  echo "$v: $(python3 -c "
import json
l=[x for x in open('gpurun_out/dpdiag.log') if x.startswith('{')][-1]
d=json.loads(l); print(d['ms_per_step'], d['config']['comm_backend'], d['config']['grad_exchange'])")"
  grep "bench.py graph" gpurun_out/dpdiag.log | cut -c1-300
done
