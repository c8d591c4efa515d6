# Development (round 6): BASELINE config 2 weak (2^28 R and S keys per rank) over 4
# rehearsal ranks on one GPU: the u16 wire reading S in place (pieces), the u16 wire with
# the round-5 gather (SGXAMD_WIRE_GATHER=1), and 4-byte keys (SGXAMD_WIRE16=0); wall
# times, then a kernel trace of each (device time = the sum of the kernels).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06j}
mkdir -p $OUT
for cfg in "pieces:" "gather:SGXAMD_WIRE_GATHER=1" "keys:SGXAMD_WIRE16=0"; do
  n=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 300 python scripts/dev/wire_time.py c2 3 4 > $OUT/c2_$n.log 2>&1 || { cat $OUT/c2_$n.log; exit 1; }
done
for cfg in "pieces:" "gather:SGXAMD_WIRE_GATHER=1" "keys:SGXAMD_WIRE16=0"; do
  n=${cfg%%:*}; e=${cfg#*:}
  [ -n "$e" ] && export $e
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$n -o kt --output-format csv -- python3 scripts/dev/wire_time.py c2 2 4 > $OUT/kt_$n.log 2>&1 || { tail $OUT/kt_$n.log; exit 1; }
  [ -n "$e" ] && unset ${e%%=*}
  find $OUT/kt_$n -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_$n.csv \;
done
cat $OUT/c2_*.log
for n in pieces gather keys; do
  python3 - $OUT/kernel_stats_$n.csv $n <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6
top = sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]
print(sys.argv[2], f"device total {tot:.2f} ms over 2 joins (+ warm-up generation)",
      [(r["Name"][:28], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1)) for r in top])
PY
done
