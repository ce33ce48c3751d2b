// pbr_census.h -- phase markers of the census builds (tools/isa_census_phases.py).
#pragma once

// Census builds (PBR_CENSUS=1, development only: tools/build_variant.sh + tools/isa_census_phases.py): PBR_PHASE marks
// where a phase of a kernel begins with an assembly comment the census tool splits the code at, fenced by scheduling
// barriers so that no instruction is scheduled across it. Product builds: nothing.
#ifndef PBR_CENSUS
#define PBR_CENSUS 0
#endif
#if PBR_CENSUS
#define PBR_PHASE(name)                          \
    do {                                         \
        __builtin_amdgcn_sched_barrier(0);       \
        asm volatile("; @phase " name);          \
        __builtin_amdgcn_sched_barrier(0);       \
    } while (0)
#else
#define PBR_PHASE(name) \
    do {                \
    } while (0)
#endif
// The start of a path the census's workload does not take (a fallback, another mode's branch): the census stops there.
#define PBR_COLD(name) PBR_PHASE("cold_" name)
