#!/bin/bash
# Development A/B builds (not part of the product): recompile the balanced-kernel translation unit
# (shade_kernels_bal.hip) -- or every kernel unit with "full" -- with extra flags and link it with the product objects
# of build/obj into abx/<name>/libpbrshade.so, for tools/ab_bench.py (PBR_LIB_PATH). Every unit compiled here is
# stamped flavor "variant: <name> <flags>" (pbr_build_info, ABI 9), so bench.py refuses the library without --dev and
# a profile of it can never pass for the product's. abx/ travels to the GPU box (it is not gpurun-ignored) and is
# deleted when the experiment is over.
#   tools/build_variant.sh NAME "-DPBR_LEAN_MIN_WAVES=5"        (run `make -C physically_based_renderer_amd/csrc` first)
#   tools/build_variant.sh NAME "" full                          (recompile every kernel unit with the flags)
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME="$1"; FLAGS="$2"; MODE="${3:-bal}"
CSRC="$ROOT/physically_based_renderer_amd/csrc"
OBJ="$ROOT/build/var/$NAME"
OUT="$ROOT/abx/$NAME"
mkdir -p "$OBJ" "$OUT"
HIPCC=/opt/rocm/bin/hipcc
SHA="$(python3 "$ROOT/physically_based_renderer_amd/_sources.py")"
FLAVOR="variant: $NAME ${FLAGS//[\"\']/}"
COMMON="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -I$ROOT/include -I$CSRC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt --offload-arch=gfx950 -munsafe-fp-atomics"
# single-quoted for the eval below, so each define keeps its double quotes (a C string) and its spaces
prov() { echo "'-DPBR_SOURCES_SHA=\"$SHA\"' '-DPBR_BUILD_FLAVOR=\"$FLAVOR\"' '-DPBR_UNIT_CFLAGS=\"$1\"'"; }
eval $HIPCC $COMMON $FLAGS $(prov "") -c "$CSRC/shade_kernels_bal.hip" -o "$OBJ/shade_kernels_bal.o"
if [ "$MODE" = full ]; then
  ILP="-mllvm -amdgpu-sched-strategy=max-ilp"
  eval $HIPCC $COMMON $FLAGS $ILP $(prov "$ILP") -c "$CSRC/shade_kernels.hip" -o "$OBJ/shade_kernels.o"
  eval $HIPCC $COMMON $FLAGS $(prov "") -c "$CSRC/pbr_context.hip" -o "$OBJ/pbr_context.o"
  K="$OBJ/shade_kernels.o"; C="$OBJ/pbr_context.o"
else
  K="$ROOT/build/obj/shade_kernels.o"; C="$ROOT/build/obj/pbr_context.o"
fi
$HIPCC --offload-arch=gfx950 -shared -o "$OUT/libpbrshade.so" "$OBJ/shade_kernels_bal.o" "$K" "$C" "$ROOT/build/obj/gbuffer_fill.o" -lpthread
echo "$OUT/libpbrshade.so"
