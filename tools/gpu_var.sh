#!/bin/bash
# radix_part run-to-run variance: R separate bench processes, buffer addresses + per-stage ms
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in $(seq 1 ${R:-6}); do
  HKCSA_CP_ADDR=1 timeout -k 10 200 python3 bench.py --steps 6 --warmup 1 --no-legs --no-cpu-baseline --patterns 0 --no-pcie > gpurun_out/var_$i.json 2> gpurun_out/var_$i.err || exit 1
  python3 - "$i" <<'PY'
import json, sys
i = sys.argv[1]
d = json.load(open(f"gpurun_out/var_{i}.json"))
st = {k: round(v["ms"] / v["launches"], 3) for k, v in d["detail"]["stages_ms_total"].items() if k.startswith("radix_part")}
addr = [l.strip() for l in open(f"gpurun_out/var_{i}.err") if l.startswith("[cp addr]")][-1]
print(i, d["ms_per_step"], st, addr)
PY
done
