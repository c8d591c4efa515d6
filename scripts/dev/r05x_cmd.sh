# Development (r05x): the u16 wire in the 8-rank rehearsal (c4), on and off, kernel traces
# of both, then (unless NOTEST) the multi-GPU test files.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05x}
mkdir -p $OUT
timeout -k 10 200 python scripts/dev/wire_time.py c4 3 > $OUT/c4_on.log 2>&1 && \
SGXAMD_WIRE16=0 timeout -k 10 200 python scripts/dev/wire_time.py c4 3 > $OUT/c4_off.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 scripts/dev/wire_time.py c4 2 > $OUT/kt.log 2>&1 && \
SGXAMD_WIRE16=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_off -o kt --output-format csv -- python3 scripts/dev/wire_time.py c4 2 > $OUT/kt_off.log 2>&1
rc=$?
if [ $rc = 0 ] && [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_multi_gpu.py tests/test_rccl_double_gpu.py 'tests/test_paths_gpu.py::test_wire16_switches' > $OUT/tests.log 2>&1
  rc=$?
  tail -3 $OUT/tests.log
fi
cat $OUT/c4_on.log $OUT/c4_off.log
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/kt_off -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_off.csv \;
exit $rc
