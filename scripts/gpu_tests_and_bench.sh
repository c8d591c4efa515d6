set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests_4.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/gpu_tests_4.log; exit 1; }
tail -3 gpurun_out/gpu_tests_4.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_1.json 2> gpurun_out/bench_1.err || { echo "bench failed"; tail -30 gpurun_out/bench_1.err; exit 1; }
cat gpurun_out/bench_1.json
lscpu > gpurun_out/lscpu.txt; nproc >> gpurun_out/lscpu.txt
