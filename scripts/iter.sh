#!/bin/bash
# Development iteration on the GPU box: parity tests, then a bench line without the
# CPU baseline.  Usage: bash scripts/iter.sh <tag> [bench args]
set -o pipefail
TAG=${1:-it}
shift || true
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1 \
  || { echo "gpu tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 600 python bench.py --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "roofline", d["roofline"]["kernel"], d["roofline"]["frac"])
print(json.dumps(d["rho"]["kernel_ms_avg"]))
sc=d.get("scan")
tp=d.get("tpch")
if tp: print("tpch SF", tp["scale_factor"], json.dumps({q: (tp[q]["ms_total_device"], tp[q]["M_rec_per_s"], tp[q]["column_GB_per_s"], tp[q]["result"]) for q in ("Q3","Q10","Q12","Q19")}))
if sc: print("scan count GB/s", sc["count"]["input_GB_per_s"], "bv", sc["bitvector"]["total_GB_per_s"], "index", sc["index"]["total_GB_per_s"], json.dumps(sc["index"]["kernel_ms_avg"]))
PY
