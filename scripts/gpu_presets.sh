# The other BASELINE configs through bench.py (c2, c4, c5), a few steps each.
set -o pipefail
mkdir -p gpurun_out
for p in c2 c4 c5; do
  timeout -k 10 300 python bench.py --preset $p --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_preset_$p.log 2>&1 || exit 1
  python3 -c "
import json
l=[x for x in open('gpurun_out/bench_preset_$p.log') if x.startswith('{')][-1]
d=json.loads(l); print('$p', round(d['ms_per_step'], 2), 'ms/step', round(d['value']), d['unit'], d['config']['launch'][:40])"
done
