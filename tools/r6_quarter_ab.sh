cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_slices.py tests/test_gpu_scale.py > gpurun_out/r6q2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6q2_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for q in main; do
    timeout -k 10 200 python3 tools/shard_emulate.py --nranks 8 --ranks 0 --pos64 > gpurun_out/r6q2_e.jsonl 2> gpurun_out/r6q2_e.err || { tail -5 gpurun_out/r6q2_e.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/r6q2_e.jsonl').readline())
print('quarter=$q rep $rep emul8', d['build_ms'], {k: v['ms_per_build'] for k,v in d['stages'].items()})"
  done
done
HKCSA_SL_TRACE=1 timeout -k 10 200 python3 tools/shard_emulate.py --nranks 8 --ranks 0 --pos64 --reps 1 2>&1 >/dev/null | grep trace | head -1
