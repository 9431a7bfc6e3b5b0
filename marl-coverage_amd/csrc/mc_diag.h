// mc_diag.h — diagnostic instrumentation of the env kernel, compiled in only
// by -DMC_STAMPS builds (tools/stamps.py): STAMP(k) records s_memtime at
// phase k of the slot's env into State::stamps [B][16].  In normal builds it
// expands to nothing.
#pragma once

#ifdef MC_STAMPS
#define STAMP(k)                                                                          \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    uint64_t _t;                                                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");            \
    if (threadIdx.x == 0 && s.stamps) s.stamps[(size_t)blockIdx.x * EPW * 16 + (k)] = _t; \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#endif
