"""Summarise the rocprofv3 PMC runs of tools/gpu_pmc.sh into profiles/pmc_kernels.json.

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes): FETCH_SIZE is in KiB and on
gfx950 reports half of the bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM), WRITE_SIZE is
exact for streaming stores.  Per bench timer name, the n-element launches of its kernel are averaged:
  sa_bucket_sort       k_bucket_sort<false, ...>          (LDS bucket sorts)
  radix_onesweep_text  k_onesweep<unsigned int, 512, 16, 0, 4, true>   (first pass, keys from text)
  radix_onesweep       k_onesweep<unsigned int, 1024, 16, 0, 4, false> (second pass)
"""
import csv, json, os, sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(root, "gpurun_out")
KERNELS = {
    "sa_bucket_sort": lambda k: "k_bucket_sort<false" in k,
    "radix_onesweep_text": lambda k: "k_onesweep<unsigned int, 512, 16, 0, 4, true" in k,
    "radix_onesweep": lambda k: "k_onesweep<unsigned int, 1024, 16, 0, 4, false" in k,
}


def per_launch(counter, match):
    rows = list(csv.DictReader(open(os.path.join(src, f"pmc_{counter}", "run_counter_collection.csv"))))
    sel = [r for r in rows if match(r["Kernel_Name"])]
    if not sel:
        return []
    gmax = max(int(r["Grid_Size"]) for r in sel)   # the n-element launches (not refinement sorts)
    return [float(r["Counter_Value"]) for r in sel if int(r["Grid_Size"]) == gmax]


out = {"note": "bench.py --steps 1 --warmup 0 --patterns 0 at 1 GiB sigma=4; per launch, KiB counters converted "
               "to GB with FETCH_SIZE doubled (gfx950 wide-read calibration)"}
for name, match in KERNELS.items():
    f, w = per_launch("FETCH_SIZE", match), per_launch("WRITE_SIZE", match)
    if not f or not w:
        continue
    rd = sum(f) * 2 * 1024 / 1e9 / len(f)
    wr = sum(w) * 1024 / 1e9 / len(w)
    out[name] = {"launches": len(f), "read_gb_per_launch": round(rd, 3), "write_gb_per_launch": round(wr, 3),
                 "traffic_gb_per_launch": round(rd + wr, 3)}
os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
json.dump(out, open(os.path.join(root, "profiles", "pmc_kernels.json"), "w"), indent=1)
print(json.dumps(out))
