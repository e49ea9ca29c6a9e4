#!/usr/bin/env python3
"""Per-kernel rocprofv3 evidence for one command: kernel-trace stats, HBM traffic and SQ counters,
each in its own pass (separate --pmc runs; rocprofv3 does not split counters over passes), keyed by
the DEMANGLED kernel name (template arguments kept, `(anonymous namespace)::` and the parameter
list dropped), so every kernel gets its own row.

usage (on the GPU box, from the repo root):
  python3 tools/kprof.py --tag r5a [--passes stats,fetch,write,sq1,sq2] [--filter REGEX] -- python3 bench.py ...
  python3 tools/kprof.py --tag r5a --summarize-only          # re-read gpurun_out/kprof_<tag>_*

Outputs:
  gpurun_out/kprof_<tag>_<pass>/run_*.csv            raw rocprofv3 output
  gpurun_out/kprof_<tag>.json                        one row per kernel and launch size
      calls, avg_us                                  (stats pass)
      read_gb, write_gb per launch                   2 x FETCH_SIZE (gfx950 reports half the bytes of wide
                                                     coalesced reads, MI355X_MICROARCH.md §HBM) and
                                                     WRITE_SIZE, KiB -> GB
      wait_any, wait_inst_any, active_inst,          fractions of SQ_WAVE_CYCLES
      wait_inst_lds
      lds_conflict                                   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
      valu_per_wave, lds_per_wave, salu_per_wave,    instructions per wave (SQ_INSTS_* / SQ_WAVES)
      vmem_rd_per_wave, vmem_wr_per_wave
      waves_per_cu                                   mean resident waves per CU over the launch
A launch size is the grid size; kernels launched at several sizes (refinement sorts) get one row per
size so the n-sized launches are not blended with small ones.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import re
import subprocess
import sys

PASSES = {
    "stats": ["--kernel-trace", "--stats"],
    "fetch": ["--pmc", "FETCH_SIZE"],
    "write": ["--pmc", "WRITE_SIZE"],
    "sq1": ["--pmc", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_WAIT_INST_LDS"],
    "sq2": ["--pmc", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
            "SQ_INSTS_VMEM_WR", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],
    "l2": ["--pmc", "TCC_HIT_sum", "TCC_MISS_sum"],
}


def kname(raw: str) -> str:
    s = raw.replace("(anonymous namespace)::", "")
    if s.startswith("void "):
        s = s[5:]
    depth = 0
    for i, ch in enumerate(s):          # cut at the parameter list: the first '(' outside template args
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return s[:i]
    return s


def run_pass(tag: str, name: str, cmd: list[str], kfilter: str | None, limit: int) -> int:
    d = f"gpurun_out/kprof_{tag}_{name}"
    args = ["timeout", "-k", "10", str(limit), "rocprofv3", *PASSES[name]]
    if kfilter and name != "stats":
        args += ["--kernel-include-regex", kfilter]
    args += ["--output-format", "csv", "-d", d, "-o", "run", "--", *cmd]
    with open(d + ".log", "w") as log:
        rc = subprocess.run(args, stdout=log, stderr=subprocess.STDOUT).returncode
    print(f"pass {name}: rc={rc}", flush=True)
    return rc


def _rows(path):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return list(csv.DictReader(f))


def summarize(tag: str) -> dict:
    rows: dict = collections.defaultdict(lambda: {"calls": 0, "dur_ns": 0.0, "ctr": collections.defaultdict(float),
                                                   "disp": collections.defaultdict(set)})
    for r in _rows(f"gpurun_out/kprof_{tag}_stats/run_kernel_trace.csv"):
        grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
        k = (kname(r["Kernel_Name"]), grid)
        rows[k]["calls"] += 1
        rows[k]["res"] = {"vgpr": int(r.get("VGPR_Count") or 0), "scratch": int(r.get("Scratch_Size") or 0),
                          "lds": int(r.get("LDS_Block_Size") or 0), "wg": int(r.get("Workgroup_Size_X") or 0)}
        rows[k]["dur_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for p in ("fetch", "write", "sq1", "sq2", "l2"):
        for r in _rows(f"gpurun_out/kprof_{tag}_{p}/run_counter_collection.csv"):
            k = (kname(r["Kernel_Name"]), int(r.get("Grid_Size", 0) or 0))
            rows[k]["ctr"][r["Counter_Name"]] += float(r["Counter_Value"])
            rows[k]["disp"][p].add(r["Dispatch_Id"])
    out = []
    for (name, grid), v in rows.items():
        c, dp = v["ctr"], v["disp"]
        row = {"kernel": name, "grid": grid, "calls": v["calls"],
               "avg_us": round(v["dur_ns"] / v["calls"] / 1e3, 2) if v["calls"] else None, **v.get("res", {})}
        if dp.get("fetch"):
            row["read_gb"] = round(2 * c["FETCH_SIZE"] * 1024 / 1e9 / len(dp["fetch"]), 4)
        if dp.get("write"):
            row["write_gb"] = round(c["WRITE_SIZE"] * 1024 / 1e9 / len(dp["write"]), 4)
        if "read_gb" in row and "write_gb" in row:
            row["traffic_gb"] = round(row["read_gb"] + row["write_gb"], 4)
            if row["avg_us"]:
                row["traffic_tbs"] = round(row["traffic_gb"] / row["avg_us"] * 1e3, 3)
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        waves = c.get("SQ_WAVES", 0.0)
        if dp.get("sq1") and wc:
            for key, ctr in (("wait_any", "SQ_WAIT_ANY"), ("wait_inst_any", "SQ_WAIT_INST_ANY"),
                             ("active_inst", "SQ_ACTIVE_INST_ANY"), ("wait_inst_lds", "SQ_WAIT_INST_LDS")):
                row[key] = round(c[ctr] / wc, 3)
            if waves:
                row["waves_per_launch"] = round(waves / len(dp["sq1"]))
                row["valu_per_wave"] = round(c["SQ_INSTS_VALU"] / waves, 1)
                row["lds_per_wave"] = round(c["SQ_INSTS_LDS"] / waves, 1)
        if dp.get("sq2"):
            if c.get("SQ_LDS_IDX_ACTIVE"):
                row["lds_conflict"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 3)
            if waves:
                row["salu_per_wave"] = round(c["SQ_INSTS_SALU"] / waves, 1)
                row["vmem_rd_per_wave"] = round(c["SQ_INSTS_VMEM_RD"] / waves, 1)
                row["vmem_wr_per_wave"] = round(c["SQ_INSTS_VMEM_WR"] / waves, 1)
            if c.get("GRBM_GUI_ACTIVE") and wc:
                # SQ_WAVE_CYCLES counts per SE in quad-cycles on CDNA; GRBM_GUI_ACTIVE in cycles per XCD
                row["waves_per_cu"] = round(wc * 4 / (c["GRBM_GUI_ACTIVE"] / 8) / 256, 2)
        if dp.get("l2") and c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0):
            row["l2_hit"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
        out.append(row)
    out.sort(key=lambda r: -(r["avg_us"] or 0) * r["calls"])
    res = {"tag": tag, "note": "per launch; read = 2 x FETCH_SIZE (gfx950 wide-read calibration), write = "
                               "WRITE_SIZE; SQ ratios are of SQ_WAVE_CYCLES; rows keyed by demangled kernel + grid",
           "kernels": out}
    with open(f"gpurun_out/kprof_{tag}.json", "w") as f:
        json.dump(res, f, indent=1)
    return res


# bench.py timer name -> kernel-name prefix (profiles/pmc_kernels.json feeds roofline.traffic)
TIMERS = {"sa_bucket_sort": "hk::k_bucket_sort_rec<", "byte_hist": "hk::k_byte_hist", "wt_bits": "hk::k_wt_bits<",
          "wt_partition": "hk::k_wt_partition<", "radix_part_text": "hk::k_cpart<0,", "radix_part": "hk::k_cpart<2,",
          "sa_bucket_hist": "hk::k_slice_hist_spans<", "fm_count": "hk::k_count<"}


def pmc_json(res: dict, path: str):
    """profiles/pmc_kernels.json: per bench timer, the HBM bytes per launch of its kernel's largest-grid row."""
    out = {"note": f"kprof {res['tag']} (bench.py --steps 1 --warmup 0 at 1 GiB sigma=4): per launch of the largest "
                   "grid, read = 2 x FETCH_SIZE (gfx950 wide-read calibration), write = WRITE_SIZE, KiB -> GB"}
    for name, pre in TIMERS.items():
        rows = [r for r in res["kernels"] if r["kernel"].startswith(pre) and "traffic_gb" in r]
        if not rows:
            continue
        r = max(rows, key=lambda x: x["grid"])
        out[name] = {"kernel": r["kernel"], "read_gb_per_launch": r["read_gb"], "write_gb_per_launch": r["write_gb"],
                     "traffic_gb_per_launch": r["traffic_gb"], "avg_us": r["avg_us"]}
        for extra in ("l2_hit", "waves_per_cu", "lds_conflict", "wait_any"):
            if extra in r:
                out[name][extra] = r[extra]
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


def main():
    argv = sys.argv[1:]
    cmd = []
    if "--" in argv:
        i = argv.index("--")
        argv, cmd = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--passes", default="stats,fetch,write,sq1,sq2,l2")
    ap.add_argument("--filter", default=None, help="kernel regex for the counter passes")
    ap.add_argument("--limit", type=int, default=240, help="seconds per pass")
    ap.add_argument("--summarize-only", action="store_true")
    ap.add_argument("--pmc-json", default=None, help="also write the bench timers' traffic (profiles/pmc_kernels.json)")
    a = ap.parse_args(argv)
    os.makedirs("gpurun_out", exist_ok=True)
    if not a.summarize_only:
        if not cmd:
            ap.error("command after -- required")
        for p in a.passes.split(","):
            rc = run_pass(a.tag, p, cmd, a.filter, a.limit)
            if rc != 0:
                print(f"pass {p} failed rc={rc}; stopping", flush=True)
                summarize(a.tag)
                sys.exit(rc)
    res = summarize(a.tag)
    if a.pmc_json:
        pmc_json(res, a.pmc_json)
    for r in res["kernels"][:40]:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
