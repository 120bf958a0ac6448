"""Per-dispatch view of rocprofv3 --pmc passes: for kernels matching FILTER,
group dispatches by (kernel, grid size) -- one group per problem size -- and
print every counter's mean per dispatch plus derived ratios.
Usage: pmc_dispatch.py DIR FILTER"""
import csv, glob, os, sys
from collections import defaultdict

root, filt = sys.argv[1], sys.argv[2]
groups = defaultdict(lambda: defaultdict(list))
order = []
for f in sorted(glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0]
        if filt not in name:
            continue
        key = (name.replace("void msp::", "")[:40], int(r["Grid_Size"]))
        if key not in groups:
            order.append(key)
        groups[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        groups[key]["_dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for key in order:
    c = {k: sum(v) / len(v) for k, v in groups[key].items()}
    out = [f"{key[0]} grid={key[1]} dur={c['_dur_ns'] / 1e3:.0f}us"]
    g = c.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back): the kernel's cycles
        # are g / 8; SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over the 1024 SIMDs (16 per 16x16x32 bf16 MFMA)
        out.append(f"mfma_busy={c['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.2f}")
        out.append(f"clk={g / 8 / c['_dur_ns']:.2f}GHz")
    if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c:
        out.append(f"lds_conflict={c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_LDS_IDX_ACTIVE'], 1):.2f}")
    if "SQ_LDS_IDX_ACTIVE" in c and g:
        out.append(f"lds_busy={c['SQ_LDS_IDX_ACTIVE'] / (g / 8 * 256):.2f}")
    if "SQ_WAIT_INST_LDS" in c and "SQ_WAVE_CYCLES" in c:
        out.append(f"wait_lds={c['SQ_WAIT_INST_LDS'] / c['SQ_WAVE_CYCLES']:.2f}")
    if "SQ_WAVES" in c and "SQ_INSTS_LDS" in c:
        out.append(f"lds/wave={c['SQ_INSTS_LDS'] / c['SQ_WAVES']:.0f}")
    if "SQ_WAVE_CYCLES" in c:
        w = c["SQ_WAVE_CYCLES"]
        out.append(f"wait_any={c['SQ_WAIT_ANY'] / w:.2f} wait_inst={c['SQ_WAIT_INST_ANY'] / w:.2f} "
                   f"active={c['SQ_ACTIVE_INST_ANY'] / w:.2f}")
    if "TCP_TCC_READ_REQ_LATENCY_sum" in c:
        out.append(f"l2_lat={c['TCP_TCC_READ_REQ_LATENCY_sum'] / max(c['TCP_TCC_READ_REQ_sum'], 1):.0f}cyc")
    if "TCP_TCC_READ_REQ_sum" in c:
        out.append(f"l2_reqs={c['TCP_TCC_READ_REQ_sum']:.3g} "
                   f"({c['TCP_TCC_READ_REQ_sum'] * 128 / (c['_dur_ns'] * 1e-9) / 1e12:.1f} TB/s at 128 B)")
    if "SQ_WAVES" in c and "SQ_INSTS_VALU" in c:
        out.append(f"valu/wave={c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.0f}")
    if "SQ_WAVES" in c and "SQ_INSTS_VMEM_RD" in c:
        out.append(f"vmem_rd/wave={c['SQ_INSTS_VMEM_RD'] / c['SQ_WAVES']:.0f}")
    if "TA_BUSY_avr" in c and g:
        out.append(f"ta_busy={c['TA_BUSY_avr'] / g:.2f}")
    if "TCC_HIT_sum" in c:
        out.append(f"l2_hit={c['TCC_HIT_sum'] / max(c['TCC_HIT_sum'] + c['TCC_MISS_sum'], 1):.2f}")
    if "FETCH_SIZE" in c:
        out.append(f"fetch={2 * c['FETCH_SIZE'] / 1e3:.0f}MB(x2)")
    if "TCP_PENDING_STALL_CYCLES_sum" in c and g:
        out.append(f"tcp_pend={c['TCP_PENDING_STALL_CYCLES_sum'] / g / 256:.2f}")
    if "TCP_TCR_TCP_STALL_CYCLES_sum" in c and g:
        out.append(f"tcr_stall={c['TCP_TCR_TCP_STALL_CYCLES_sum'] / g / 256:.2f}")
    print(" ".join(out))
