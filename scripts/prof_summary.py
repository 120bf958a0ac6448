"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"{'kernel':70s} {'calls':>6s} {'total ms':>9s} {'%':>5s} {'avg us':>8s}")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    name = r['Name'].split('(')[0][:70]
    print(f"{name:70s} {r['Calls']:>6s} {float(r['TotalDurationNs'])/1e6:9.2f} {100*float(r['TotalDurationNs'])/tot:5.1f} {float(r['AverageNs'])/1e3:8.1f}")
print(f"total kernel time {tot/1e6:.1f} ms")
# the conv family (one msp_conv_tile / msp_conv_nbr call = one conv kernel + its
# split_weights [+ split_reduce]): average per call, to set beside bench.py's
# roofline.avg_launch_us (HIP events around each call)
fam = ("conv_x6g_kernel", "conv_x6r_kernel", "conv_x6d_kernel", "conv_x6p_kernel", "conv_tile7_kernel",
       "conv_tilep_kernel", "conv_tile4_kernel", "conv_tile_kernel", "conv_x6s_kernel", "conv_x6l_kernel")
ft = sum(float(r['TotalDurationNs']) for r in rows if any(c in r['Name'] for c in fam + ("split_weights_kernel", "split_weights_lane_kernel", "split_reduce_kernel")))
fn = sum(int(r['Calls']) for r in rows if any(c + '<' in r['Name'] or c + '(' in r['Name'] for c in fam))
if fn:
    print(f"conv family: {fn} calls, {ft / fn / 1e3:.1f} us per call (kernel + split_weights + split_reduce)")
