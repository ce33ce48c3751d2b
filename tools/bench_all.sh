#!/bin/bash
# One bench line per BASELINE config and mode on the gpurun box:
#   tools/bench_all.sh <out.jsonl>
# Each run is its own process under its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out="${1:-gpurun_out/bench_all.jsonl}"
mkdir -p "$(dirname "$out")"
: > "$out"
for spec in "3 faithful" "3 exact" "2 faithful" "2 exact" "4 faithful" "4 exact" "1 faithful" "1 exact"; do
  set -- $spec
  echo "=== config $1 mode $2"
  timeout -k 10 240 python3 bench.py --config "$1" --mode "$2" --no-cpu-baseline >> "$out" 2> "${out%.jsonl}_cfg$1_$2.err" || exit $?
  tail -n 1 "$out" | cut -c1-200
done
