#!/bin/bash
# Round 4: the fused slice pass A (one T' scan per group of 4 slices) + the faster cursor pre-pass:
# slice / bucket parity, the strong 4 GiB N = 1 line, the 4 GiB single-handle tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_slices.py tests/test_gpu_bucket.py > gpurun_out/r4i_quick.log 2>&1
rc=$?; tail -3 gpurun_out/r4i_quick.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --strong --steps 3 --warmup 1 > gpurun_out/r4i_strong.json 2> gpurun_out/r4i_strong.err || exit $?
python3 -c "
import json;d=json.loads(open('gpurun_out/r4i_strong.json').read());st=d['detail']['stages_ms_total']
print('strong', d['ms_per_step'], {k: round(v['ms']/d['steps'],3) for k,v in st.items()})"
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py -k "single_handle" > gpurun_out/r4i_scale.log 2>&1
rc=$?; tail -3 gpurun_out/r4i_scale.log; exit $rc
