#!/bin/bash
# A/B of library variants on one box: LIBS="base new" (hkcsa/_lib/libhkcsa_<name>.so; "main" = libhkcsa.so),
# alternating runs of the 1 GiB sigma=4 bench (SA + BWT steps only), per-kernel averages printed.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib
for rep in ${REPS:-1 2}; do
  for v in ${LIBS:-base main}; do
    lib=$L/libhkcsa_$v.so; [ "$v" = main ] && lib=$L/libhkcsa.so
    HKCSA_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup 5 --no-legs --no-cpu-baseline \
      --no-eps --no-pcie --no-harness --patterns 0 > gpurun_out/ab_${v}_$rep.json 2> gpurun_out/ab_${v}_$rep.err || exit $?
    python3 -c "
import json;d=json.loads(open('gpurun_out/ab_${v}_$rep.json').read());st=d['detail']['stages_ms_total']
print('$v rep $rep', d['ms_per_step'], {k: round(v['ms']/d['steps'],3) for k,v in st.items() if v['ms']/d['steps'] > 0.2})"
  done
done
