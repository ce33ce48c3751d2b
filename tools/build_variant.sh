#!/bin/bash
# Development A/B builds (not part of the product): recompile only the balanced-kernel translation unit
# (shade_kernels_bal.hip) with extra flags and link it with the product objects of build/obj into
# abx/<name>/libpbrshade.so, for tools/ab_bench.py (PBR_LIB_PATH). abx/ travels to the GPU box (it is not
# gpurun-ignored) and is deleted when the experiment is over.
#   tools/build_variant.sh NAME "-DPBR_BAL_EXPERIMENT=1"       (run `make -C physically_based_renderer_amd/csrc` first)
#   tools/build_variant.sh NAME "" full                          (recompile every kernel TU with the flags)
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME="$1"; FLAGS="$2"; MODE="${3:-bal}"
CSRC="$ROOT/physically_based_renderer_amd/csrc"
OBJ="$ROOT/build/var/$NAME"
OUT="$ROOT/abx/$NAME"
mkdir -p "$OBJ" "$OUT"
HIPCC=/opt/rocm/bin/hipcc
COMMON="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -I$ROOT/include -I$CSRC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt --offload-arch=gfx950 -munsafe-fp-atomics"
$HIPCC $COMMON $FLAGS -c "$CSRC/shade_kernels_bal.hip" -o "$OBJ/shade_kernels_bal.o"
if [ "$MODE" = full ]; then
  $HIPCC $COMMON $FLAGS -mllvm -amdgpu-sched-strategy=max-ilp -c "$CSRC/shade_kernels.hip" -o "$OBJ/shade_kernels.o"
  $HIPCC $COMMON $FLAGS -c "$CSRC/pbr_context.hip" -o "$OBJ/pbr_context.o"
  K="$OBJ/shade_kernels.o"; C="$OBJ/pbr_context.o"
else
  K="$ROOT/build/obj/shade_kernels.o"; C="$ROOT/build/obj/pbr_context.o"
fi
$HIPCC --offload-arch=gfx950 -shared -o "$OUT/libpbrshade.so" "$OBJ/shade_kernels_bal.o" "$K" "$C" "$ROOT/build/obj/gbuffer_fill.o" -lpthread
echo "$OUT/libpbrshade.so"
