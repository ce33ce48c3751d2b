#!/bin/bash
# Collect the round's rocprofv3 evidence on the gpurun box:
#   1. --kernel-trace --stats of the default bench command (the bench line's own run);
#   2. separate --pmc passes (never combined with other traces): FETCH_SIZE, WRITE_SIZE, SQ
#      instruction / cycle counters, on a short bench run of the same workload.
# Output: gpurun_out/prof_<tag>/...; tools/pmc_summarize.py turns it into profiles/.
# usage: tools/profile_round.sh <tag> [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tag="$1"; shift
out="gpurun_out/prof_$tag"
mkdir -p "$out"
run() {  # name, timeout, command...
  local name="$1" tmo="$2"; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$tmo" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "$out/$name.log"
  return $rc
}
run kt 300 rocprofv3 --kernel-trace --stats -d "$out/kt" -o kt --output-format csv -- python3 bench.py "$@" &&
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$out/pmc_fetch" -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 1 --ramp-ms 0 --no-cpu-baseline "$@" &&
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$out/pmc_write" -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 1 --ramp-ms 0 --no-cpu-baseline "$@" &&
run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$out/pmc_sq" -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 1 --ramp-ms 0 --no-cpu-baseline "$@" &&
run pmc_busy 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d "$out/pmc_busy" -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 1 --ramp-ms 0 --no-cpu-baseline "$@"
