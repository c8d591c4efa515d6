# Development: A/B of library variants (varlib/<name>) on the config-3 scans, alternating, twice.
# Usage (through gpurun): VARIANTS="head other" bash scripts/dev/scan_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/scan_ab
for rep in 1 2; do for v in ${VARIANTS:-head}; do
  SGXAMD_LIB_PATH=$PWD/varlib/$v/libsgxamd.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-tpch --no-cpu-baseline --no-paper --no-configs --no-tuple-layout > gpurun_out/scan_ab/$v.$rep.json 2> gpurun_out/scan_ab/$v.$rep.err || { tail -5 gpurun_out/scan_ab/$v.$rep.err; exit 1; }
  python3 -c "
import json; s=json.load(open('gpurun_out/scan_ab/$v.$rep.json'))['scan']
print('$v', $rep, s['count']['kernel_ms_avg'], s['bitvector']['kernel_ms_avg'], s['index']['kernel_ms_avg'])"
done; done
