"""Per-kernel SQ counter summary of tools/gpu_pmc2.sh passes: per-dispatch-averaged wait / issue
fractions, VALU and LDS instructions per wave, bank-conflict share, resident waves per CU."""
import collections, csv, re, glob, json, os, sys

src = sys.argv[1]
out = {}
for tag in sys.argv[2:]:
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    nd = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(src, f"{tag}_*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"^void |hk::|\(anonymous namespace\)::", "", r["Kernel_Name"])
            k = re.sub(r"\(.*", "", k)[:90]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            nd[k].add((f, r["Dispatch_Id"]))
    for k, t in tot.items():
        wc = t["SQ_WAVE_CYCLES"] or 1
        w = t["SQ_WAVES"] or 1
        g = t["GRBM_GUI_ACTIVE"]
        out[f"{tag}:{k}"] = {
            "dispatches": len(nd[k]) // 2,
            "valu_per_wave": round(t["SQ_INSTS_VALU"] / w), "salu_per_wave": round(t["SQ_INSTS_SALU"] / w),
            "lds_per_wave": round(t["SQ_INSTS_LDS"] / w), "vmem_rd_per_wave": round(t["SQ_INSTS_VMEM_RD"] / w),
            "wait_any": round(t["SQ_WAIT_ANY"] / wc, 3), "wait_inst_any": round(t["SQ_WAIT_INST_ANY"] / wc, 3),
            "active_inst": round(t["SQ_ACTIVE_INST_ANY"] / wc, 3), "active_valu": round(t["SQ_ACTIVE_INST_VALU"] / wc, 3),
            "wait_inst_lds": round(t["SQ_WAIT_INST_LDS"] / wc, 3),
            "lds_conflict": round(t["SQ_LDS_BANK_CONFLICT"] / max(t["SQ_LDS_IDX_ACTIVE"], 1), 3),
            "waves_per_cu": round(wc * 4 / (g / 8) / 256, 2) if g else None,
            "valu_busy_frac_per_simd": round(t["SQ_ACTIVE_INST_VALU"] * 4 / (g / 8) / 1024, 3) if g else None,
        }
print(json.dumps(out, indent=1))
