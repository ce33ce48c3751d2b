#!/bin/bash
# Where the shading kernel's waves wait (development tool): one --pmc pass of 8 SQ counters per config -- the
# instruction counts and in-flight levels of scalar (SMEM: light records), vector (VMEM: G-buffer, env map) and
# LDS instructions next to SQ_WAIT_ANY and SQ_WAVE_CYCLES. LEVEL / INSTS is the mean latency of that kind in
# cycles (MI355X_MICROARCH.md, SQ counters). Output: gpurun_out/wait_c<N>[_<mode>]/; tools/wait_summary.py reads it.
# usage (on the gpurun box): tools/wait_pmc.sh <config> <mode> [<config> <mode> ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS"
while [ $# -ge 2 ]; do
  c=$1; m=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/wait_c${c}_$m -o pmc --output-format csv -- \
    python3 bench.py --config $c --mode $m --steps 5 --warmup 1 --ramp-ms 0 --no-cpu-baseline --no-anchor > gpurun_out/wait_c${c}_$m.log 2>&1 || exit $?
done
