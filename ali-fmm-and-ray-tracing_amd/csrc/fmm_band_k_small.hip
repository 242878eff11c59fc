// fmm_band_k_small.hip — fmm_band_k.hip built for short band steps: 256-thread members (one wave
// per SIMD, so the registers of a whole SIMD lane — no spills), the sort buckets and fallback rounds
// sized to 4 waves.  The host launches it (af_launch_band_k_small) when a source has many members
// and each member's lists are short (option "small_members").
#define AF_BAND_SMALL 1
#define AF_THREADS 256
#define AF_WPE_N 1
#define AF_SORTB 256
#define AF_FB_ROUND 64
#include "fmm_band_k.hip"
