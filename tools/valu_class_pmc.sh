#!/bin/bash
# Dynamic VALU instruction classes of one bench workload: two --pmc passes of 8 SQ counters each
# (never combined with traces), on a short bench run. Output: gpurun_out/vclass_<tag>/{a,b}/...; summarised by
# tools/valu_class_summary.py. usage (on the gpurun box): tools/valu_class_pmc.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tag="$1"; shift
out="gpurun_out/vclass_$tag"
mkdir -p "$out"
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
B="SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F64"
timeout -s KILL 120 rocprofv3 --pmc $A -d "$out/a" -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 1 --ramp-ms 0 --no-cpu-baseline --no-anchor "$@" > "$out/a.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $B -d "$out/b" -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 1 --ramp-ms 0 --no-cpu-baseline --no-anchor "$@" > "$out/b.log" 2>&1
