#!/bin/bash
# Per-wave stall breakdown of the shading kernel (development tool): one --pmc pass of 8 SQ counters per
# config on a short bench run (no other trace domains). WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY
# ~= WAVE_CYCLES (MI355X_MICROARCH.md, SQ counters). Output: gpurun_out/stall_c<N>/.
# usage (on the gpurun box): tools/stall_pmc.sh [configs...]   (default: 2 3 4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES"
for c in ${@:-2 3 4}; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/stall_c$c -o pmc --output-format csv -- \
    python3 bench.py --config $c --steps 5 --warmup 1 --ramp-ms 0 --no-cpu-baseline > gpurun_out/stall_c$c.log 2>&1 || exit $?
done
