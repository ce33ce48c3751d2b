#!/bin/bash
# Instruction counts of development builds (not part of the product): one --pmc pass of 8 SQ counters per library
# in abx/<name>/ on one bench config, so the VALU / SALU / LDS instructions per wave of each experiment build can be
# set side by side (tools/variant_summary.py). Output: gpurun_out/vpmc_<name>/.
# usage (on the gpurun box): tools/variant_pmc.sh <config> <mode> <name> [<name> ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD"
cfg=$1; mode=$2; shift 2
for v in "$@"; do
  PBR_LIB_PATH="$PWD/abx/$v/libpbrshade.so" timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/vpmc_$v -o pmc \
    --output-format csv -- python3 bench.py --config $cfg --mode $mode --steps 5 --warmup 1 --ramp-ms 0 \
    --no-cpu-baseline --no-anchor > gpurun_out/vpmc_$v.log 2>&1 || exit $?
  echo "vpmc $v done"
done
