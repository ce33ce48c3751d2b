#!/usr/bin/env python3
"""oracle/strip_hlsl.py -- TEST INFRASTRUCTURE ONLY (builds the checker, never the product).

A syntax-only transform that lets g++ compile the reference's own pixel-shader text as C++:

    /root/reference/Source/Shaders/Core.hlsl      -> oracle/_ref/gen/Core.hlsl
    /root/reference/Source/Shaders/Default.hlsl   -> oracle/_ref/gen/Default.hlsl      (PS as shipped)
                                                   -> oracle/_ref/gen/Default_ibl.hlsl  (the IBL block revived)
    /root/reference/Source/Shaders/Skybox.hlsl    -> oracle/_ref/gen/Skybox.hlsl

LightingUtil.hlsl needs no transform: Core.hlsl's `#include "LightingUtil.hlsl"` resolves to the
reference file itself (the Makefile puts /root/reference/Source/Shaders on the include path).
Output goes only to oracle/_ref/ (git-ignored); nothing of the reference is committed.

Every rewrite is a change of *syntax* that C++ needs, and each one is counted: the script fails if a
rule does not fire the expected number of times, so a changed reference text cannot slip through
silently. The arithmetic, the operation order, the control flow and the permutation `#if`s are the
reference's own text.

  rule                                    HLSL (reference)                        C++ (generated)
  register bindings                       `: register(t0)`                        removed
  cbuffer blocks  (Core.hlsl:28,35,64)    `cbuffer cbPass : register(b1) {`       `inline namespace cbPass {`
  cbuffer / resource storage              `float3 g_CameraPosW;`                  `PBR_HLSL_GLOBAL float3 g_CameraPosW;`
                                                                                 (thread_local: one set of constants
                                                                                  per harness thread)
  vertex semantics                        `float3 PosW : POSITION;`               `float3 PosW;`
  render-target semantic                  `float4 PS(VertexOut pin) : SV_Target`  `float4 PS(VertexOut pin)`
  swizzles                                `.xyz .xy .xyww .rgb .r`                 `.xyz() .xy() .xyww() .rgb() .r()`
  zero-initialising cast                  `(VertexOut)0.0f`                       `VertexOut{}`
  cbuffer light capacity (Core.hlsl:60)   `Light g_Lights[MAX_LIGHTS];`           `... g_Lights[PBR_ORACLE_MAX_LIGHTS];`

The capacity rule is the one non-syntactic edit: MAX_LIGHTS (LightingUtil.hlsl:7) is 16, and BASELINE
configs run 64 and 256 lights; a D3D12 build of the reference would need the same edit (a cbuffer
holds up to 4096 float4s = 1365 lights). `ComputeLighting`'s `Light gLights[MAX_LIGHTS]` parameter
decays to a pointer in C++ and is untouched.

Default_ibl.hlsl is the IBL_DIFFUSE variant: the author's commented-out block
Default.hlsl:140-149 with its comment markers removed, and line 150 (the constant ambient it was
replaced by) commented out -- exactly what re-enabling the block in the reference takes.

usage: strip_hlsl.py <reference Shaders dir> <output dir>
"""
from __future__ import annotations

import os
import re
import sys


def _sub(pattern: str, repl, text: str, expect: int | None, what: str, flags: int = 0) -> str:
    out, n = re.subn(pattern, repl, text, flags=flags)
    if expect is not None and n != expect:
        raise SystemExit(f"strip_hlsl: rule '{what}' fired {n} times, expected {expect}")
    return out


def _storage_in_cbuffers(text: str) -> tuple[str, int]:
    """`cbuffer X {` -> `namespace X {` and prefix every member declaration with PBR_HLSL_GLOBAL."""
    out, pos, blocks = [], 0, 0
    for m in re.finditer(r"\bcbuffer\s+(\w+)\s*\{", text):
        out.append(text[pos:m.start()])
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(text[i], 0)
            i += 1
        body = text[m.end():i - 1]
        body = re.sub(r"(?m)^([ \t]*)(?=[A-Za-z_]\w*\s+[A-Za-z_]\w*\s*(\[[^\]]*\])?\s*;)", r"\1PBR_HLSL_GLOBAL ", body)
        out.append(f"inline namespace {m.group(1)} {{{body}}}")
        pos, blocks = i, blocks + 1
    out.append(text[pos:])
    return "".join(out), blocks


def common(text: str, name: str) -> str:
    """The rules every file gets (counts are per file, see EXPECT)."""
    e = EXPECT[name]
    text = _sub(r"\s*:\s*register\(\s*\w+\s*\)", "", text, e["register"], "register bindings")
    text, nb = _storage_in_cbuffers(text)
    if nb != e["cbuffer"]:
        raise SystemExit(f"strip_hlsl: {name}: {nb} cbuffer blocks, expected {e['cbuffer']}")
    text = _sub(r"(?m)^([ \t]*)(?=(Texture2D|SamplerState)\s)", r"\1PBR_HLSL_GLOBAL ", text, e["resources"],
                "resource storage")
    text = _sub(r"(\w+)\s*:\s*(POSITION|NORMAL|TANGENT|BINORMAL|TEXCOORD|SV_POSITION)\s*;", r"\1;", text,
                e["semantics"], "vertex semantics")
    text = _sub(r"\)\s*:\s*SV_Target", ")", text, e["sv_target"], "render-target semantic")
    text = _sub(r"\.(xyww|xyz|xy|rgb|r)\b(?!\s*\()", r".\1()", text, e["swizzles"], "swizzles")
    text = _sub(r"\((\w+)\)\s*0\.0f", r"\1{}", text, e["zero_cast"], "zero-initialising cast")
    text = _sub(r"\bg_Lights\[MAX_LIGHTS\]", "g_Lights[PBR_ORACLE_MAX_LIGHTS]", text, e["capacity"],
                "cbuffer light capacity")
    return text


def revive_ibl(text: str) -> str:
    """Default.hlsl:139-150: un-comment the IBL block, comment out the constant-ambient line."""
    pat = (r"(// ambient lighting solved wih the IBL\s*\n)\s*/\*\s*\n(.*?float3 litColor = ambient \+ directLight;"
           r"[^\n]*\n)\s*\*/\s*\n(\s*)(float3 litColor = g_AmbientLight \* diffuseAlbedo \+ directLight;)")
    return _sub(pat, r"\1\n\2\n\3// \4  (replaced by the block above)", text, 1, "IBL block", flags=re.S)  # same line count


# Expected rule counts per file, read off the reference text (Core.hlsl:16-80, Default.hlsl:1-161,
# Skybox.hlsl:1-49). Swizzles in Default.hlsl: .xyz (28), .xy (42), .rgb (80, 92, 105, 144, 160), .r (86, 99,
# 112), plus .r (57) and .xy (62) inside the commented-out displacement block; Skybox.hlsl: .xyz (29),
# .xyww (32), .rgb (48).
EXPECT = {
    "Core.hlsl": dict(register=11, cbuffer=3, resources=8, semantics=0, sv_target=0, swizzles=0, zero_cast=0,
                      capacity=1),
    "Default.hlsl": dict(register=0, cbuffer=0, resources=0, semantics=11, sv_target=1, swizzles=12, zero_cast=1,
                         capacity=0),
    "Skybox.hlsl": dict(register=0, cbuffer=0, resources=0, semantics=7, sv_target=1, swizzles=3, zero_cast=0,
                        capacity=0),
}

HEADER = ("// GENERATED by oracle/strip_hlsl.py from {src} -- syntax-only transform of the reference's shader\n"
          "// text for the C++ oracle build (TEST INFRASTRUCTURE; git-ignored, never committed).\n"
          "#line 1 \"{src}\"\n")  # diagnostics and __LINE__ keep the reference's own line numbers


def main(argv: list[str]) -> int:
    if len(argv) != 3:
        print(__doc__.strip().splitlines()[-1], file=sys.stderr)
        return 2
    src_dir, out_dir = argv[1], argv[2]
    os.makedirs(out_dir, exist_ok=True)
    outputs = {}
    for name in ("Core.hlsl", "Default.hlsl", "Skybox.hlsl"):
        path = os.path.join(src_dir, name)
        with open(path, encoding="utf-8") as f:
            text = f.read().replace("\r\n", "\n")
        outputs[name] = (path, common(text, name))
    outputs["Default_ibl.hlsl"] = (outputs["Default.hlsl"][0], revive_ibl(outputs["Default.hlsl"][1]))
    for name, (src, text) in outputs.items():
        with open(os.path.join(out_dir, name), "w", encoding="utf-8") as f:
            f.write(HEADER.format(src=src) + text)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
