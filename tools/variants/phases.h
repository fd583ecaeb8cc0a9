// Phase markers for tools/isa_phases.py (static per-phase instruction budgets): compile a unit with
//   hipcc ... -include tools/variants/phases.h --save-temps
// and the kernels' NNGP_PHASE(name) points become scheduling barriers around a named asm comment.
#pragma once
#define NNGP_PHASE(name)                        \
    __builtin_amdgcn_sched_barrier(0);          \
    asm volatile("; PHASE_" #name ::: "memory"); \
    __builtin_amdgcn_sched_barrier(0)
