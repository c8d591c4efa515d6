cd sgxv2-analytical-query-processing-benchmarks_amd/tools || exit 1
export TMPDIR=/tmp
timeout -k 5 60 ./bw_lab 31 g || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d ../../gpurun_out/half -o f --output-format csv -- ./bw_lab 31 g > /dev/null 2>&1 || exit 1
