"""HBM traffic per msp_conv_tile call from rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE in separate runs, MI355X_MICROARCH.md's
HBM/rocprofv3 section): FETCH_SIZE is doubled (gfx950 tallies 128-B
requests at 64 B), WRITE_SIZE taken as is; both are in KB per dispatch.

One conv-family call (msp_conv_local / msp_conv_tile / msp_conv_nbr) launches one conv kernel (conv_x6s /
conv_x6l / conv_x6d / conv_x6r / conv_x6g, older forms conv_x6p / conv_tilep / conv_tile7 / conv_tile4 /
conv_tile) plus a split_weights(_lane) and, for split grids, a split_reduce; traffic per call = sum
over the family's dispatches / number of conv kernel dispatches.
Writes JSON: python scripts/pmc_traffic.py gpurun_out/pmc_<tag> out.json"""
import csv, glob, json, os, sys

root, out_path = sys.argv[1], sys.argv[2]
conv_names = ("conv_x6s_kernel", "conv_x6l_kernel", "conv_x6d_kernel", "conv_x6p_kernel", "conv_x6r_kernel", "conv_x6g_kernel", "conv_tile7_kernel", "conv_tilep_kernel", "conv_tile4_kernel", "conv_tile_kernel")
tot = {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0}
by_kernel = {}  # short kernel name -> {counter: total KB x 1024, dispatches}
ndisp = {"FETCH_SIZE": 0, "WRITE_SIZE": 0}
dur = {"FETCH_SIZE": 0, "WRITE_SIZE": 0}
for f in sorted(glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        ctr = r["Counter_Name"]
        if ctr not in tot:
            continue
        is_conv = any(c + "<" in name or c + "(" in name for c in conv_names)
        short = name.split("(")[0].replace("void ", "").replace("msp::", "")
        k = by_kernel.setdefault(short, {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0, "n_FETCH_SIZE": 0, "n_WRITE_SIZE": 0})
        k[ctr] += float(r["Counter_Value"]) * 1024.0
        k["n_" + ctr] += 1
        if is_conv or "split_reduce_kernel" in name or "split_weights_kernel" in name or "split_weights_lane_kernel" in name:
            tot[ctr] += float(r["Counter_Value"]) * 1024.0
            if is_conv:
                ndisp[ctr] += 1
                dur[ctr] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
fetch = 2.0 * tot["FETCH_SIZE"] / max(ndisp["FETCH_SIZE"], 1)
write = tot["WRITE_SIZE"] / max(ndisp["WRITE_SIZE"], 1)
res = {"kernel": "msp_conv_local / msp_conv_tile / msp_conv_nbr", "calls": ndisp["FETCH_SIZE"],
       "fetch_bytes_per_call": fetch, "write_bytes_per_call": write, "traffic_bytes_per_call": fetch + write,
       "note": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) and WRITE_SIZE in separate runs of "
               "`bench.py --steps 2 --warmup 1 --no-cpu`; conv kernel + split_weights(_lane) + split_reduce dispatches per call"}
# per kernel (every kernel of the run): bytes per dispatch and the share of the conv family's traffic
fam = {}
for short, k in by_kernel.items():
    n = max(k["n_FETCH_SIZE"], k["n_WRITE_SIZE"], 1)
    f, w = 2.0 * k["FETCH_SIZE"], k["WRITE_SIZE"]
    fam[short] = {"dispatches": n, "fetch_bytes_per_dispatch": f / max(k["n_FETCH_SIZE"], 1),
                  "write_bytes_per_dispatch": w / max(k["n_WRITE_SIZE"], 1),
                  "fetch_bytes_per_conv_call": f / max(ndisp["FETCH_SIZE"], 1),
                  "write_bytes_per_conv_call": w / max(ndisp["WRITE_SIZE"], 1)}
res["by_kernel"] = dict(sorted(fam.items(), key=lambda kv: -(kv[1]["fetch_bytes_per_conv_call"] +
                                                             kv[1]["write_bytes_per_conv_call"])))
json.dump(res, open(out_path, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != 'by_kernel'}, indent=1))
for kk, vv in list(res['by_kernel'].items())[:25]:
    print(f"{vv['fetch_bytes_per_conv_call'] / 1e6:9.2f} {vv['write_bytes_per_conv_call'] / 1e6:9.2f} MB per conv call  {vv['dispatches']:6d}  {kk}")
