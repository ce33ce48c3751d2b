// pbr_build_info.h -- what each compilation unit of libpbrshade.so was built from (pbr_build_info, ABI 9).
//
// The Makefile compiles every unit with
//   PBR_SOURCES_SHA  the stamp of the checkout's sources (physically_based_renderer_amd/_sources.py: sha256 of
//                    csrc/*, the Makefile and the public header), the key of committed profiles;
//   PBR_BUILD_FLAVOR "product" for the default target without EXTRA flags; "debug_bounds", "asan",
//                    "custom: <EXTRA>" or "variant: <name> <flags>" (tools/build_variant.sh) otherwise;
//   PBR_UNIT_CFLAGS  the unit's own extra compiler flags (e.g. the max-ILP scheduler of shade_kernels.hip).
// PBR_UNIT_INFO(name, switches) forms the unit's JSON record; each unit defines one C symbol with it at its end,
// and pbr_build_info (pbr_context.hip) lists them all, so bench.py and the profile tools can tell the library a
// process LOADED from the sources in the checkout, and refuse a development or stale build.
#pragma once

#ifndef PBR_SOURCES_SHA
#define PBR_SOURCES_SHA "unstamped"
#endif
#ifndef PBR_BUILD_FLAVOR
#define PBR_BUILD_FLAVOR "unstamped"
#endif
#ifndef PBR_UNIT_CFLAGS
#define PBR_UNIT_CFLAGS ""
#endif

#define PBR_BI_STR2(x) #x
#define PBR_BI_STR(x) PBR_BI_STR2(x)
// One build switch as a JSON member: "NAME": "value as the preprocessor sees it".
#define PBR_BI_SWITCH(name) "\"" #name "\": \"" PBR_BI_STR(name) "\""

#define PBR_UNIT_INFO(unit, switches)                                                                  \
    "{\"unit\": \"" unit "\", \"sources_sha\": \"" PBR_SOURCES_SHA "\", \"flavor\": \"" PBR_BUILD_FLAVOR \
    "\", \"cflags\": \"" PBR_UNIT_CFLAGS "\", \"switches\": {" switches "}}"
