"""Summarise a tools/gpu_profile_r2.sh run into profiles/ (tracked evidence for the bench line).

usage: python tools/profile_summary.py [gpurun_out] [tag]

Legs of one bench.py run are told apart by the k_synth dispatch that creates each synthetic text:
leg 0 = the headline (1 GiB sigma=4), leg 1 = sigma=256 (1 GiB), leg 2 = printable 200 MiB.

Outputs (tag default r2):
  profiles/<tag>_kernel_stats.csv   per leg and kernel: calls, total / avg / min / max us (kernel trace)
  profiles/pmc_kernels.json         HBM traffic per launch of the roofline kernels (sigma=4 at the top
                                    level, sigma=256 under "sigma256"): 2*FETCH_SIZE + WRITE_SIZE, KiB ->
                                    GB (FETCH_SIZE doubled: gfx950 reports half of the bytes of wide
                                    streaming reads, MI355X_MICROARCH.md §HBM)
  profiles/<tag>_sq_counters.json   SQ issue / LDS counters per kernel (leg 0, n-sized launches)
  profiles/<tag>_count_pmc.json     L2 hit rate and occupancy of k_count per leg
"""
import collections
import csv
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
TAG = sys.argv[2] if len(sys.argv) > 2 else "r2"
PROF = os.path.join(ROOT, "profiles")
LEGS = ["sigma4", "sigma256", "printable_200MiB"]

# bench timer name -> kernel-name predicate (the n-sized launches are the largest grids)
TIMERS = {
    # k_onesweep<V, T, I, MODE, LBW, FT, LB>: FT = the text pass (keys built from the text)
    "sa_bucket_sort": lambda k: "k_bucket_sort_fast<" in k or "k_bucket_sort<false" in k,
    "radix_onesweep_text": lambda k: "k_onesweep<" in k and ", true, " in k,
    "radix_onesweep": lambda k: "k_onesweep<" in k and ", false, " in k,
    "byte_hist": lambda k: "k_byte_hist" in k,
    "wt_bits": lambda k: "k_wt_bits" in k,
    "wt_partition": lambda k: "k_wt_partition" in k,
    # k_cpart<MODE, LB, NB, T>: MODE 0 = pass A from the text, 1 = pass A from packed keys, 2 = pass B
    "radix_part_text": lambda k: "k_cpart<0," in k,
    "radix_part_keys": lambda k: "k_cpart<1," in k,
    "radix_part": lambda k: "k_cpart<2," in k,
    "sa_bucket_hist": lambda k: "k_bucket_hist_spans" in k or "k_slice_hist_spans" in k,
    "sa_digit_hist": lambda k: "k_bucket_hist<" in k,
    "fm_count": lambda k: "k_count" in k,
}


def short(name: str) -> str:
    name = name.replace("hk::(anonymous namespace)::", "")
    return name.split("(")[0] if "(" in name and "<" not in name.split("(")[0] else name[:120]


def kernel_trace(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    out, leg = [], -1
    for name, st, en in rows:
        if "k_synth" in name:
            leg += 1
        out.append((max(leg, 0), name, (en - st) / 1000.0))
    return out


def stats_csv(trace, path):
    agg = collections.OrderedDict()
    for leg, name, us in trace:
        k = (LEGS[leg] if leg < len(LEGS) else f"leg{leg}", short(name))
        agg.setdefault(k, []).append(us)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["leg", "kernel", "calls", "total_us", "avg_us", "min_us", "max_us"])
        for (leg, name), v in sorted(agg.items(), key=lambda kv: (kv[0][0], -sum(kv[1]))):
            w.writerow([leg, name, len(v), round(sum(v), 2), round(sum(v) / len(v), 3), round(min(v), 3),
                        round(max(v), 3)])


def pmc_rows(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    leg, out, seen = -1, [], set()
    for r in rows:
        if "k_synth" in r["Kernel_Name"] and r["Dispatch_Id"] not in seen:   # one row per counter
            seen.add(r["Dispatch_Id"])
            leg += 1
        r["leg"] = max(leg, 0)
        out.append(r)
    return out


def per_launch(rows, counter, match, leg):
    sel = [r for r in rows if r["leg"] == leg and r["Counter_Name"] == counter and match(r["Kernel_Name"])]
    if not sel:
        return []
    gmax = max(int(r["Grid_Size"]) for r in sel)
    per = collections.defaultdict(float)
    for r in sel:
        if int(r["Grid_Size"]) == gmax:
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(per.values())


def main():
    os.makedirs(PROF, exist_ok=True)
    db = os.path.join(SRC, f"{TAG}_stats", "run_results.db")
    if os.path.exists(db):
        stats_csv(kernel_trace(db), os.path.join(PROF, f"{TAG}_kernel_stats.csv"))
    fetch = os.path.join(SRC, f"{TAG}_pmc_FETCH_SIZE", "run_counter_collection.csv")
    write = os.path.join(SRC, f"{TAG}_pmc_WRITE_SIZE", "run_counter_collection.csv")
    if os.path.exists(fetch) and os.path.exists(write):
        fr, wr = pmc_rows(fetch), pmc_rows(write)
        out = {"note": f"bench.py --steps 1 --warmup 0 (round {TAG}); per n-sized launch: read = 2 x FETCH_SIZE "
                       "(gfx950 wide-read calibration), write = WRITE_SIZE, KiB -> GB"}
        for leg, key in ((0, None), (1, "sigma256")):
            d = {}
            for name, match in TIMERS.items():
                f, w = per_launch(fr, "FETCH_SIZE", match, leg), per_launch(wr, "WRITE_SIZE", match, leg)
                if not f or not w:
                    continue
                rd = sum(f) * 2 * 1024 / 1e9 / len(f)
                wb = sum(w) * 1024 / 1e9 / len(w)
                d[name] = {"launches": len(f), "read_gb_per_launch": round(rd, 3), "write_gb_per_launch": round(wb, 3),
                           "traffic_gb_per_launch": round(rd + wb, 3)}
            if key:
                out[key] = d
            else:
                out.update(d)
        json.dump(out, open(os.path.join(PROF, "pmc_kernels.json"), "w"), indent=1)
    sq = {}
    for i in (1, 2):
        p = os.path.join(SRC, f"{TAG}_sq_{i}", "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        rows = pmc_rows(p)
        for name, match in TIMERS.items():
            for r in rows:
                if r["leg"] != 0 or not match(r["Kernel_Name"]):
                    continue
            ctrs = sorted({r["Counter_Name"] for r in rows if r["leg"] == 0 and match(r["Kernel_Name"])})
            for c in ctrs:
                v = per_launch(rows, c, match, 0)
                if v:
                    sq.setdefault(name, {})[c] = sum(v) / len(v)
    for name, d in sq.items():
        if "SQ_WAVE_CYCLES" in d:
            wc = d["SQ_WAVE_CYCLES"]
            d["frac_wait_any"] = round(d.get("SQ_WAIT_ANY", 0) / wc, 4)
            d["frac_wait_inst_any"] = round(d.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
            d["frac_active_inst"] = round(d.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)
            d["frac_wait_inst_lds"] = round(d.get("SQ_WAIT_INST_LDS", 0) / wc, 4)
        if "SQ_LDS_IDX_ACTIVE" in d and d["SQ_LDS_IDX_ACTIVE"]:
            d["lds_bank_conflict_frac"] = round(d.get("SQ_LDS_BANK_CONFLICT", 0) / d["SQ_LDS_IDX_ACTIVE"], 4)
        if "GRBM_GUI_ACTIVE" in d and "SQ_WAVE_CYCLES" in d:
            # resident waves per CU: wave-quad-cycles x 4 over (per-XCD GPU cycles x 256 CUs)
            d["mean_waves_per_cu"] = round(d["SQ_WAVE_CYCLES"] * 4 / (d["GRBM_GUI_ACTIVE"] / 8) / 256, 2)
    if sq:
        sq["note"] = ("leg 0 (1 GiB sigma=4), n-sized launches, averaged per launch; SQ_WAVE_CYCLES / SQ_WAIT_* / "
                      "SQ_ACTIVE_* in quad-cycles; mean_waves_per_cu uses GRBM_GUI_ACTIVE of set 2 with the wave "
                      "cycles of set 1 (separate passes of the same launch)")
        json.dump(sq, open(os.path.join(PROF, f"{TAG}_sq_counters.json"), "w"), indent=1)
    p = os.path.join(SRC, f"{TAG}_count", "run_counter_collection.csv")
    if os.path.exists(p):
        rows = pmc_rows(p)
        res = {}
        for leg in sorted({r["leg"] for r in rows}):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in rows:
                if r["leg"] == leg and "k_count" in r["Kernel_Name"]:
                    per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            if not per:
                continue
            tot = collections.defaultdict(float)
            for d in per.values():
                for k, v in d.items():
                    tot[k] += v
            hit, miss = tot.get("TCC_HIT_sum", 0), tot.get("TCC_MISS_sum", 0)
            e = {"launches": len(per), "l2_hit_rate": round(hit / (hit + miss), 4) if hit + miss else None}
            if tot.get("GRBM_GUI_ACTIVE"):
                e["mean_waves_per_cu"] = round(tot["SQ_WAVE_CYCLES"] * 4 / (tot["GRBM_GUI_ACTIVE"] / 8) / 256, 2)
                e["max_waves_per_cu"] = 32
                e["occupancy"] = round(e["mean_waves_per_cu"] / 32, 4)
            e.update({k: v / len(per) for k, v in tot.items()})
            res[LEGS[leg] if leg < len(LEGS) else f"leg{leg}"] = e
        res["note"] = "k_count (batched backward search): sigma4 = 1M x 16-symbol, printable_200MiB = 1M x 20-symbol"
        json.dump(res, open(os.path.join(PROF, f"{TAG}_count_pmc.json"), "w"), indent=1)
    print("written to", PROF)


if __name__ == "__main__":
    main()
