cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r5w TESTS="tests/test_gpu_english.py tests/test_gpu_parity.py::test_sa_bwt_wt_vs_oracle tests/test_gpu_slices.py" STEPS="quick" bash tools/gpu_suite.sh || exit $?
for lg in english english; do
  echo "== $lg"
  timeout -k 10 400 python3 -u bench.py --only-leg $lg --leg-steps 3 > gpurun_out/r5w_$lg.json 2> gpurun_out/r5w_$lg.err || exit $?
  python3 - gpurun_out/r5w_$lg.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st=d["stages_ms_total"]; k=d["steps"]
print(d["ms_per_step"], d.get("tied_after_round")[:6], {a: round(v["ms"]/k,2) for a,v in st.items() if v["ms"]/k > 0.4})
PY
done
HKCSA_X=1 TAG=r5w STEPS="profen" bash tools/gpu_suite.sh || exit $?
