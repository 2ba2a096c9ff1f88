// diag.h -- diagnostics hooks of the kernels (timing ablations and per-wave phase stamps).
//
// In the release build every hook is a no-op: DBG(x) is 0, DIAG / PH / BPH expand to nothing and
// no stamp storage or diagnostics entry point exists, so the kernels compile exactly as if the
// hooks were absent.  Diagnostics builds define
//   -DBE_DIAG_SKIP    DBG(x) reads KParams::dbg (BALLENV_DEBUG_SKIP): skip / early-exit bits
//   -DBE_DIAG_STAMPS  the above plus per-wave stamps (s_memrealtime / s_memtime) into device
//                     tables, read back through be_diag_stamps / be_board_diag_stamps
// (tools/build_diag.sh, tools/build_ab_lib.sh; tools/stamps.hip, tools/*_phases.py read them).
// Outputs of a diagnostics build are wrong whenever a skip bit is set.
//
// A translation unit selects its section before including: BE_DIAG_UNIT_STEP (csrc/ballenv.hip,
// inside its anonymous namespace) or BE_DIAG_UNIT_BOARD (csrc/board.hip); each unit then expands
// its BE_DIAG_*_ENTRIES macro inside its extern "C" block.
#pragma once

#if defined(BE_DIAG_UNIT_STEP)
// phase-skip bits (DBG): tools/ablate.py, tools/fused_ablate.py, tools/policy_ablate.py
enum : uint32_t { DBG_NO_STATS = 1, DBG_NO_RASTER = 2, DBG_NO_OBS = 4, DBG_NO_PHILOX = 8, DBG_NO_DYN = 16,
                  DBG_NO_NEAR = 32, DBG_EXIT_ENTRY = 64, DBG_EXIT_BARRIER = 128, DBG_EXIT_PHYSICS = 256,
                  DBG_EXIT_RASTER = 512, DBG_WAIT_LOADS = 1024,
                  // fused policy rollout: every env on the table / no select_action tail / no block barriers
                  DBG_POL_TABLE = 2048, DBG_POL_NO_FINISH = 4096, DBG_POL_NO_SYNC = 8192,
                  DBG_NO_RESET = 16384, DBG_NO_COPY = 32768 };
#if defined(BE_DIAG_STAMPS) || defined(BE_DIAG_SKIP)
#define DBG(x) (p.dbg & (x))
#else
#define DBG(x) 0
#endif

#ifdef BE_DIAG_STAMPS
// DIAG(pt): per-wave stamp `pt` of a one-step kernel; PH_INIT / PH(k) / PH_STORE: per-phase cycle
// accumulators of a multi-step kernel (PH(k) adds the cycles since the previous PH to phase k,
// PH_STORE writes them to g_diag_cy[wave][k])
constexpr int DIAG_WAVES = 1 << 16, DIAG_POINTS = 16;
__device__ unsigned long long g_diag_rt[DIAG_WAVES][DIAG_POINTS];   // s_memrealtime (100 MHz, chip-wide)
__device__ unsigned long long g_diag_cy[DIAG_WAVES][DIAG_POINTS];   // s_memtime (shader clock)
__device__ unsigned int g_diag_hw[DIAG_WAVES];                       // HW_ID (cu/sh/se) | XCC_ID << 28
__device__ __forceinline__ void diag_stamp(int point) {
  const int w = (int)(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
  if (point == 0 && (threadIdx.x & 63) == 0 && w < DIAG_WAVES)
    g_diag_hw[w] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) & 0x0FFFFFFFu |
                   ((unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 28);
  if ((threadIdx.x & 63) == 0 && w < DIAG_WAVES) {
    g_diag_rt[w][point] = __builtin_amdgcn_s_memrealtime();
    g_diag_cy[w][point] = __builtin_amdgcn_s_memtime();
  }
}
#define DIAG(pt) diag_stamp(pt)
#define PH_INIT unsigned long long ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ph_t = __builtin_amdgcn_s_memtime()
#define PH(k) do { const unsigned long long ph_n = __builtin_amdgcn_s_memtime(); ph_acc[k] += ph_n - ph_t; ph_t = ph_n; } while (0)
#define PH_STORE do { \
    const int ph_w = (int)(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64); \
    if ((threadIdx.x & 63) == 0 && ph_w < DIAG_WAVES) \
      for (int ph_k = 0; ph_k < 8; ++ph_k) g_diag_cy[ph_w][ph_k] = ph_acc[ph_k]; \
  } while (0)
// C entries (expanded in ballenv.hip's extern "C" block): the stamp tables, DIAG_WAVES x DIAG_POINTS
#define BE_DIAG_STEP_ENTRIES                                                                          \
  int be_diag_stamps(unsigned long long* rt, unsigned long long* cy) {                               \
    if (hipMemcpyFromSymbol(rt, HIP_SYMBOL(g_diag_rt), sizeof(g_diag_rt)) != hipSuccess) return BE_E_HIP; \
    if (hipMemcpyFromSymbol(cy, HIP_SYMBOL(g_diag_cy), sizeof(g_diag_cy)) != hipSuccess) return BE_E_HIP; \
    return BE_OK;                                                                                     \
  }                                                                                                   \
  int be_diag_hwid(unsigned int* hw) {                                                                \
    return hipMemcpyFromSymbol(hw, HIP_SYMBOL(g_diag_hw), sizeof(g_diag_hw)) == hipSuccess ? BE_OK : BE_E_HIP; \
  }                                                                                                   \
  int be_diag_clear(void) {                                                                           \
    static unsigned long long zero[DIAG_WAVES][DIAG_POINTS];                                          \
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_diag_rt), zero, sizeof(zero)) != hipSuccess) return BE_E_HIP;  \
    return BE_OK;                                                                                     \
  }
#else
#define DIAG(pt) ((void)0)
#define PH_INIT ((void)0)
#define PH(k) ((void)0)
#define PH_STORE ((void)0)
#define BE_DIAG_STEP_ENTRIES
#endif
#endif  // BE_DIAG_UNIT_STEP

#if defined(BE_DIAG_UNIT_BOARD)
#ifdef BE_DIAG_STAMPS
// per-wave cycles per phase of the createBoard kernels (s_memtime deltas summed over a launch):
// BPH(k) closes phase k; BCOUNT(k, v) adds a count (slots 5..7), read with be_board_diag_stamps
constexpr int BDIAG_WAVES = 1 << 14;
__device__ unsigned long long g_bdiag[BDIAG_WAVES][8];
#define BPH_INIT unsigned long long bph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, bph_t = __builtin_amdgcn_s_memtime()
#define BPH(k) do { const unsigned long long bph_n = __builtin_amdgcn_s_memtime(); bph_acc[k] += bph_n - bph_t; bph_t = bph_n; } while (0)
#define BCOUNT(k, v) (bph_acc[k] += (unsigned long long)(v))
#define BPH_STORE do { \
    const int bph_w = (int)(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64); \
    if ((threadIdx.x & 63) == 0 && bph_w < BDIAG_WAVES) \
      for (int bph_k = 0; bph_k < 8; ++bph_k) g_bdiag[bph_w][bph_k] = bph_acc[bph_k]; \
  } while (0)
#define BE_DIAG_BOARD_ENTRIES                                                                          \
  int be_board_diag_stamps(unsigned long long* cy) {                                                  \
    return hipMemcpyFromSymbol(cy, HIP_SYMBOL(g_bdiag), sizeof(g_bdiag)) == hipSuccess ? BE_OK : BE_E_HIP; \
  }
#else
#define BPH_INIT ((void)0)
#define BPH(k) ((void)0)
#define BCOUNT(k, v) ((void)0)
#define BPH_STORE ((void)0)
#define BE_DIAG_BOARD_ENTRIES
#endif
#endif  // BE_DIAG_UNIT_BOARD
