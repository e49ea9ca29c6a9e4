"""Summarise the rocprofv3 PMC runs of tools_gpu_pmc.sh into profiles/pmc_radix_onesweep.json.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE is in KiB and on gfx950
reports half of the bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM), WRITE_SIZE is exact
for streaming stores.  Only the large-sort launches (k_onesweep<*, 512, 16, ...>) are averaged."""
import csv, json, os, sys

root = os.path.dirname(os.path.abspath(__file__))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(root, "gpurun_out")


def per_launch(counter):
    rows = list(csv.DictReader(open(os.path.join(src, f"pmc_{counter}", "run_counter_collection.csv"))))
    sel = [r for r in rows if "k_onesweep" in r["Kernel_Name"] and ", 512, 16," in r["Kernel_Name"]]
    gmax = max(int(r["Grid_Size"]) for r in sel)          # the n-element passes of the main sort
    return [float(r["Counter_Value"]) for r in sel if int(r["Grid_Size"]) == gmax]


f, w = per_launch("FETCH_SIZE"), per_launch("WRITE_SIZE")
# the first pass of the sort reads no values (iota), later passes read keys + values
out = {
    "kernel": "k_onesweep<unsigned int, 512, 16, 0, 4> (radix_onesweep)",
    "launches": len(f),
    "fetch_kib": f, "write_kib": w,
    "traffic_gb_per_launch": round(sum(2 * a + b for a, b in zip(f, w)) * 1024 / 1e9 / max(1, len(f)), 3),
    "read_gb_per_launch_corrected": round(sum(f) * 2 * 1024 / 1e9 / max(1, len(f)), 3),
    "write_gb_per_launch": round(sum(w) * 1024 / 1e9 / max(1, len(w)), 3),
    "note": "bench.py --steps 1 --warmup 0 --patterns 0 at 1 GiB sigma=4; FETCH_SIZE doubled per the gfx950 "
            "calibration for wide reads (keys are read 8 B/lane, values 4 B/lane: uncalibrated widths)",
}
os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
json.dump(out, open(os.path.join(root, "profiles", "pmc_radix_onesweep.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if not k.endswith("kib")}))
