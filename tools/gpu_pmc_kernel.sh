#!/bin/bash
# SQ / LDS counters of one kernel (regex $1) over a short bench run, two passes (<= 8 SQ counters
# each); output under gpurun_out/pmc_<tag>_{1,2}.  Usage: bash tools/gpu_pmc_kernel.sh REGEX TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-legs --patterns 0"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "$1" --output-format csv \
      -d gpurun_out/pmc_$2_$i -o run -- $B > gpurun_out/pmc_$2_$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc_$2_$i.log; exit 1; }
done
python3 - "$2" <<'PY'
import csv, collections, sys
tag = sys.argv[1]
tot = collections.defaultdict(float); disp = set()
for i in (1, 2):
    for r in csv.DictReader(open(f"gpurun_out/pmc_{tag}_{i}/run_counter_collection.csv")):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add((i, r["Dispatch_Id"]))
wc = tot["SQ_WAVE_CYCLES"] or 1
print({k: round(v) for k, v in tot.items()})
print({"dispatches": len(disp) // 2, "wait_any": round(tot["SQ_WAIT_ANY"] / wc, 3), "wait_inst_any": round(tot["SQ_WAIT_INST_ANY"] / wc, 3),
       "active_inst": round(tot["SQ_ACTIVE_INST_ANY"] / wc, 3), "wait_inst_lds": round(tot["SQ_WAIT_INST_LDS"] / wc, 3),
       "lds_conflict": round(tot["SQ_LDS_BANK_CONFLICT"] / max(tot["SQ_LDS_IDX_ACTIVE"], 1), 3),
       "waves_per_cu": round(tot["SQ_WAVE_CYCLES"] * 4 / (tot["GRBM_GUI_ACTIVE"] / 8) / 256, 2) if tot["GRBM_GUI_ACTIVE"] else None})
PY
