#!/bin/bash
# GPU-box check of the pipelined join and the multi-rank path on one GPU:
# the new GPU tests, then bench.py under torchrun with 2 gloo ranks sharing cuda:0.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${1:-dist}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_rho_gpu.py tests/test_dist_gpu.py tests/test_scan_gpu.py > "$OUT/tests.log" 2>&1 \
  || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --log2n 26 --dist-backend gloo \
  > "$OUT/bench2.json" 2> "$OUT/bench2.err" || { echo "bench2 failed"; tail -30 "$OUT/bench2.err"; exit 1; }
cat "$OUT/bench2.json"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-tpch --no-cpu-baseline > "$OUT/bench1.json" 2> "$OUT/bench1.err" \
  || { echo "bench1 failed"; tail -30 "$OUT/bench1.err"; exit 1; }
cat "$OUT/bench1.json"
