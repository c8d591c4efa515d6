# Development (r05y): BASELINE config 2 weak (2^28 R and S keys per rank) over 4 rehearsal
# ranks on one GPU, the u16 wire (default mode) on and off, with kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05y}
mkdir -p $OUT
timeout -k 10 300 python scripts/dev/wire_time.py c2 3 4 > $OUT/c2_on.log 2>&1 && \
SGXAMD_WIRE16=0 timeout -k 10 300 python scripts/dev/wire_time.py c2 3 4 > $OUT/c2_off.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 scripts/dev/wire_time.py c2 2 4 > $OUT/kt.log 2>&1 && \
SGXAMD_WIRE16=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_off -o kt --output-format csv -- python3 scripts/dev/wire_time.py c2 2 4 > $OUT/kt_off.log 2>&1
rc=$?
cat $OUT/c2_on.log $OUT/c2_off.log
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/kt_off -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_off.csv \;
exit $rc
