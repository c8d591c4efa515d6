# Development: config-1 small-join timing with an environment switch on and off,
# alternating, twice.  Usage (through gpurun): bash scripts/dev/c1_env_ab.sh <tag> <VAR> "<values>"
set -o pipefail
TAG=$1; VAR=$2; VALS=$3
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for v in $VALS; do
    echo -n "$VAR=$v " >> "$OUT/c1_ab.log"
    env "$VAR=$v" timeout -k 10 120 python scripts/dev/c1_time.py 300 >> "$OUT/c1_ab.log" 2>&1 \
      || { echo "c1 $v failed"; tail -20 "$OUT/c1_ab.log"; exit 1; }
  done
done
cat "$OUT/c1_ab.log"
