#!/bin/bash
# rocprofv3 kernel stats of the 1 GiB bench with an env toggle on / off (AB_VAR=NAME).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in 1 0; do
  export $AB_VAR=$v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pab_$v -o run -- python3 bench.py --steps 10 --warmup 2 --no-legs --no-cpu-baseline --no-pcie > gpurun_out/pab_$v.json 2> gpurun_out/pab_$v.err || { tail -5 gpurun_out/pab_$v.err; exit 1; }
  f=$(find gpurun_out/pab_$v -name "run_kernel_stats.csv" | sort | tail -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
print("AB", sys.argv[2])
for x in sorted(r, key=lambda x: -float(x["TotalDurationNs"]))[:8]:
    print(" ", x["Name"][:60], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), round(float(x["MinNs"]) / 1e3, 1), round(float(x["MaxNs"]) / 1e3, 1))
PY
done
