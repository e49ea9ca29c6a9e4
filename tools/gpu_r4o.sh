#!/bin/bash
# Round 4: the strong 4 GiB N = 1 build's wall time per call against its kernel time, main vs c1 (round-4
# pre-refinement library), then the strong bench line with main.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib
for v in main c1; do
  lib=$L/libhkcsa_$v.so; [ "$v" = main ] && lib=$L/libhkcsa.so
  HKCSA_LIB=$lib timeout -k 10 400 python3 -u tools/strong_probe.py > gpurun_out/r4o_probe_$v.log 2>&1
  rc=$?; echo "$v"; cat gpurun_out/r4o_probe_$v.log | grep build; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -u bench.py --strong --steps 3 --warmup 1 > gpurun_out/r4o_strong.json 2> gpurun_out/r4o_strong.err || exit $?
python3 -c "
import json;d=json.loads(open('gpurun_out/r4o_strong.json').read());print('strong', d['ms_per_step'])"
