// Diagnostic build only (-DWF_STAMPS, waafle_amd/build.py build(stamps=True)): shader-clock
// laps per phase of the kernels, read by scripts/wave_stamps.py through the
// wf_stamps_read_<tag> / wf_stamps_reset_<tag> entry points.  The product build compiles
// every macro below to nothing (and exports no stamp entry points).  Included by
// wf_device.h inside namespace wf { namespace { } }.
//   STAMP / LAP / STAT        staged workgroup kernels (thread 0; g_stamps)
//   WLAP / WSTAT              the first wave form, every 16th contig (g_wstamps;
//                             -DWF_STAMPS_ROLL=1: the roll-up launches instead of level 0)
//   TLAP                      the level-0 triage, every 16th contig (g_tstamps)
//   SLAP / SSTAT              sp_two, every 8th contig (g_sstamps)
//   BLAP / BSTAT              sp_level (k_big_sparse, k_dump_sparse<0>), every 8th (g_bstamps)
#pragma once
#ifdef WF_STAMPS
#ifndef WF_STAMPS_ROLL
#define WF_STAMPS_ROLL 0
#endif
#define WF_STAMPS_ONLY(...) __VA_ARGS__
// extern "C" readers of one translation unit's lap array (outside the anonymous namespace)
#define WF_STAMP_READER(tag, arr, n)                                                          \
  extern "C" int wf_stamps_read_##tag(unsigned long long* out, int m) {                       \
    if (m > (n)) m = (n);                                                                     \
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(arr), sizeof(unsigned long long) * m) == hipSuccess ? 0 : -2; \
  }                                                                                           \
  extern "C" int wf_stamps_reset_##tag(void) {                                                \
    unsigned long long z[n] = {0};                                                            \
    return hipMemcpyToSymbol(HIP_SYMBOL(arr), z, sizeof z) == hipSuccess ? 0 : -2;            \
  }
__device__ unsigned long long g_stamps[32];
__shared__ unsigned long long g_tlast;   // thread 0's last stamp (workgroup-local)
#define STAMP_INIT() do { if (threadIdx.x == 0) g_tlast = __builtin_amdgcn_s_memtime(); } while (0)
#define STAMP(i)                                                                    \
  do {                                                                              \
    if (threadIdx.x == 0) {                                                         \
      unsigned long long now_ = __builtin_amdgcn_s_memtime();                       \
      atomicAdd(&g_stamps[i], now_ - g_tlast);                                      \
      g_tlast = now_;                                                               \
    }                                                                               \
  } while (0)
#define STAMP_SYNC() __syncthreads()
// wave-0 lap timer inside a phase (no barrier): cycles since the last LAP_MARK/LAP
#define LAP_MARK() unsigned long long lap_ = __builtin_amdgcn_s_memtime()
#define LAP(i)                                                                      \
  do {                                                                              \
    unsigned long long n_ = __builtin_amdgcn_s_memtime();                           \
    if (threadIdx.x == 0) atomicAdd(&g_stamps[i], n_ - lap_);                       \
    lap_ = n_;                                                                      \
  } while (0)
#define LAP_WAIT_LDS() __builtin_amdgcn_s_waitcnt(0xc07f)
#define LAP_WAIT_V(v) asm volatile("" ::"v"(v))
#define STAT(i, v) do { if (threadIdx.x == 0) atomicAdd(&g_stamps[i], (unsigned long long)(v)); } while (0)
__device__ unsigned long long g_wstamps[48];
#define WLAP_MARK() unsigned long long wlap_ = __builtin_amdgcn_s_memtime(); const bool wsamp_ = !FULL && (WF_STAMPS_ROLL ? ROLL : !ROLL) && (c & 15) == 0
#define WLAP(i)                                                                     \
  do {                                                                              \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime();                     \
    if (wsamp_ && lane == 0) atomicAdd(&g_wstamps[i], n_ - wlap_);                  \
    wlap_ = n_;                                                                     \
  } while (0)
#define WSTAT(i, v) do { if (wsamp_ && lane == 0) atomicAdd(&g_wstamps[i], (unsigned long long)(v)); } while (0)
__device__ unsigned long long g_tstamps[16];
#define TLAP_MARK() unsigned long long tlap_ = __builtin_amdgcn_s_memtime(); const bool tsamp_ = (c & 15) == 0
#define TLAP(i)                                                                     \
  do {                                                                              \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime();                     \
    if (tsamp_ && lane == 0) atomicAdd(&g_tstamps[i], n_ - tlap_);                  \
    tlap_ = n_;                                                                     \
  } while (0)
__device__ unsigned long long g_sstamps[16];
#define SLAP_MARK(c) unsigned long long slap_ = __builtin_amdgcn_s_memtime(); const bool ssamp_ = ((c) & 7) == 0
#define SLAP(i)                                                                     \
  do {                                                                              \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime();                     \
    if (ssamp_ && (threadIdx.x & 63) == 0) atomicAdd(&g_sstamps[i], n_ - slap_);    \
    slap_ = n_;                                                                     \
  } while (0)
#define SSTAT(i, v) do { if (ssamp_ && (threadIdx.x & 63) == 0) atomicAdd(&g_sstamps[i], (unsigned long long)(v)); } while (0)
// ... and of sp_level (k_big_sparse, k_dump_sparse<0>) on every 8th contig
// (slots 0-23 every contig-level; 24-33 the phases again for roll-up levels >= 1 alone, 34
// their sampled count; `level` is sp_level's)
__device__ unsigned long long g_bstamps[48];
#define BLAP_MARK(c) unsigned long long blap_ = __builtin_amdgcn_s_memtime(); const bool bsamp_ = ((c) & 7) == 0
#define BLAP(i)                                                                     \
  do {                                                                              \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime();                     \
    if (bsamp_ && (threadIdx.x & 63) == 0) {                                        \
      atomicAdd(&g_bstamps[i], n_ - blap_);                                         \
      if (level > 0) atomicAdd(&g_bstamps[24 + (i)], n_ - blap_);                   \
    }                                                                               \
    blap_ = n_;                                                                     \
  } while (0)
#define BSTAT(i, v) do { if (bsamp_ && (threadIdx.x & 63) == 0) atomicAdd(&g_bstamps[i], (unsigned long long)(v)); } while (0)
#else
#define WF_STAMPS_ONLY(...)
#define WF_STAMP_READER(tag, arr, n)
#define STAMP_INIT() do {} while (0)
#define STAMP(i) do {} while (0)
#define STAMP_SYNC() do {} while (0)
#define LAP_MARK() do {} while (0)
#define LAP(i) do {} while (0)
#define LAP_WAIT_LDS() do {} while (0)
#define LAP_WAIT_V(v) do {} while (0)
#define STAT(i, v) do {} while (0)
#define WLAP_MARK() do {} while (0)
#define WLAP(i) do {} while (0)
#define WSTAT(i, v) do {} while (0)
#define TLAP_MARK() do {} while (0)
#define TLAP(i) do {} while (0)
#define BLAP_MARK(c) do {} while (0)
#define BLAP(i) do {} while (0)
#define BSTAT(i, v) do {} while (0)
#define SLAP_MARK(c) do {} while (0)
#define SLAP(i) do {} while (0)
#define SSTAT(i, v) do {} while (0)
#endif
