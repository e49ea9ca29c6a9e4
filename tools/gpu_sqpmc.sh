#!/bin/bash
# SQ counters (issue / wait / LDS) of selected kernels during one 1 GiB bench step, one rocprofv3
# --pmc pass per counter set.  usage: KRE="regex" [SQCMD="python3 ..."] bash tools/gpu_sqpmc.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
KRE=${KRE:-"bucket_sort|bucket_hist"}
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "$KRE" --output-format csv \
      -d gpurun_out/sqpmc_$i -o run -- ${SQCMD:-python3 bench.py --steps 1 --warmup 0 --patterns 0 --no-cpu-baseline} \
      > gpurun_out/sqpmc_$i.log 2>&1
  rc=$?
  echo "set $i rc=$rc"; tail -2 gpurun_out/sqpmc_$i.log
  [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/sqpmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-60:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {v:.4g}")
PY
