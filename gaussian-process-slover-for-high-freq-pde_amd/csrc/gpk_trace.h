// gpk_trace.h — device-side timeline probes for latency tuning (build: `make trace`, which
// defines GPK_TRACE and writes libgpk_trace.so; the product build compiles them away).
//
// Every translation unit owns two slot arrays (first arrival / last departure, read from the
// 100 MHz constant clock, s_memrealtime) and exposes them to gpk_api.cpp through
// trace_fetch_<tu> / trace_reset_<tu>.  Slots are global across TUs (see SLOT_* below), so
// one step's timeline is the union of all TUs' arrays.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gpk {

constexpr int TRACE_SLOTS = 256;
enum TraceSlot {
  SLOT_CLASS_EVAL = 0, SLOT_GATHER = 1, SLOT_PIVOT0_WAIT = 2, SLOT_PIVOT0 = 3,
  SLOT_SWEEP = 4,         // + k (k < 16): whole sweep launch k
  SLOT_SWEEP_PIVOT = 20,  // + k: the next-pivot factorisation inside sweep k
  SLOT_PREFETCH_MISS = 36,  // chain, factor 0: first / last pivot whose inputs missed the prefetch
  SLOT_PG_GARR = 37,        // pgrad tail: a group's last block arrived (first / last group)
  SLOT_PG_ULAST = 38,       // pgrad U plane: the last U workgroup done
  SLOT_CLASS_SUM = 40, SLOT_PGRAD = 41, SLOT_PG_CONTRACT = 42, SLOT_PG_GROUP = 43,
  SLOT_PG_TOP = 44, SLOT_PG_UPLANE = 45, SLOT_PG_FINAL = 46,
  // dispatch spread (last workgroup start) and intermediate points
  SLOT_PG_START = 47, SLOT_PG_STAGED = 48, SLOT_CSUM_START = 49, SLOT_CEVAL_START = 50,
  SLOT_GATHER_START = 51, SLOT_CSUM_LOADED = 52, SLOT_CHAIN_END = 53, SLOT_CHAIN_M1 = 54,
  // chain, last sweep, tile (T-1, T-1) of factor 0: L^{-1} flag seen, L^{-1} in LDS, products
  // done, outputs stored + done-counter returned; 62: the same end point, last aug tile
  SLOT_LAST_FLAG = 58, SLOT_LAST_LDS = 59, SLOT_LAST_MMA = 60, SLOT_LAST_OUT = 61, SLOT_LAST_AUG = 62,
  SLOT_GEMM = 64,  // + 4 * stage: first wg [start, end], + 1: first wg operands loaded,
                   // + 2: first wg MFMAs done, + 3: last wg [start, end]  (stages < 16)
  // chain_multi_kernel, factor 0, sweep k < 16, the workgroup owning tile (k+2, k+2) (the pivot
  // chain's next-but-one input): + k
  SLOT_MC_PANEL = 128,  // panel tiles waited for and loads issued
  SLOT_MC_PIV = 144,    // L_k^{-1} flag seen
  SLOT_MC_LDS = 160,    // L_k^{-1} and panel tiles in LDS
  SLOT_MC_V = 176,      // V products stored to LDS
  SLOT_MC_PUB = 192,    // the pass-0 tiles published (flags raised)
  SLOT_MC_DONE = 208,   // pass 1 done (end of the sweep)
  SLOT_MC_PROD = 224,   // pass-0 products done (before their stores)
  // chain_multi_kernel, factor 0, sweep k < 16, every workgroup publishing panel row k + 1:
  // [first, last] inputs (panel + L_k^{-1}) in, [first, last] pass 0 published.  These reuse the
  // GEMM-stage and 128-wide-update slots, which a 1D (chain_multi) step never fires
  SLOT_MCP_IN = 64, SLOT_MCP_OUT = 240,
  // ... the last inputs-in and the last publication as (clock << 16 | blockIdx.x); the pivot
  // chain's workgroup id (mpos)
  SLOT_MCP_WHO_IN = 80, SLOT_MCP_WHO_OUT = 96, SLOT_MCP_MPOS = 112,
  // wide_update_kernel (spdinv_big.hip), sweep BIG_PROBE_SWEEP, factor 0: launch start (first
  // workgroup), pivot workgroup [start, its tile done], pivot128 done, panel workgroups [first
  // start, L^{-1} seen], panel done (last), tile workgroups' round 0 / 1 ends (max), quarter
  // items [first start, last end]
  SLOT_BIG_START = 240, SLOT_BIG_PIVTILE = 241, SLOT_BIG_PIVOT = 242, SLOT_BIG_PANEL_WAIT = 243,
  SLOT_BIG_PANEL = 244, SLOT_BIG_ROUND0 = 245, SLOT_BIG_ROUND1 = 246, SLOT_BIG_QUARTER = 247,
  // rounds 0 and 1 of the tile workgroups (+ 3 j): [first, last] start, first K-step's MFMAs done
  // (the base loads waited for), K-loop done (before the stores)
  SLOT_BIG_R0START = 248,
};
constexpr int BIG_PROBE_SWEEP = 8;

#ifdef GPK_TRACE
#define GPK_TRACE_TU(tu)                                                                  \
  namespace {                                                                             \
  __device__ unsigned long long trace_lo[TRACE_SLOTS], trace_hi[TRACE_SLOTS];             \
  }                                                                                       \
  void trace_fetch_##tu(uint64_t* lo, uint64_t* hi) {                                     \
    (void)hipMemcpyFromSymbol(lo, HIP_SYMBOL(trace_lo), sizeof(trace_lo));                \
    (void)hipMemcpyFromSymbol(hi, HIP_SYMBOL(trace_hi), sizeof(trace_hi));                \
  }                                                                                       \
  void trace_reset_##tu() {                                                               \
    unsigned long long lo[TRACE_SLOTS], hi[TRACE_SLOTS];                                  \
    for (int i = 0; i < TRACE_SLOTS; ++i) lo[i] = ~0ull, hi[i] = 0ull;                    \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(trace_lo), lo, sizeof(lo));                        \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(trace_hi), hi, sizeof(hi));                        \
  }
// probes fire in thread 0 of ONE workgroup per slot (a first-block / last-block / critical
// block); same-address atomics from every workgroup would serialise and distort the timeline
#define TR_FIRST (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0)
#define TR_LAST                                                                       \
  (threadIdx.x == 0 && blockIdx.x == gridDim.x - 1 && blockIdx.y == gridDim.y - 1 && \
   blockIdx.z == gridDim.z - 1)
#define TR_LO(slot) atomicMin(&trace_lo[slot], (unsigned long long)wall_clock64())
#define TR_HI(slot) atomicMax(&trace_hi[slot], (unsigned long long)wall_clock64())
// the LAST arriving workgroup's id: (clock << 16 | id) under atomicMax (decoded by tools/timeline.py)
#define TR_WHO(slot, id) atomicMax(&trace_hi[slot], ((unsigned long long)wall_clock64() << 16) | (unsigned)(id))
#else
#define GPK_TRACE_TU(tu)                                   \
  void trace_fetch_##tu(uint64_t* lo, uint64_t* hi) {      \
    for (int i = 0; i < TRACE_SLOTS; ++i) lo[i] = hi[i] = 0; \
  }                                                        \
  void trace_reset_##tu() {}
#define TR_FIRST false
#define TR_LAST false
#define TR_LO(slot) ((void)0)
#define TR_HI(slot) ((void)0)
#define TR_WHO(slot, id) ((void)0)
#endif

void trace_fetch_assemble(uint64_t* lo, uint64_t* hi);
void trace_reset_assemble();
void trace_fetch_spdinv(uint64_t* lo, uint64_t* hi);
void trace_reset_spdinv();
void trace_fetch_pgrad(uint64_t* lo, uint64_t* hi);
void trace_reset_pgrad();
void trace_fetch_gemm(uint64_t* lo, uint64_t* hi);
void trace_reset_gemm();
void trace_fetch_spdbig(uint64_t* lo, uint64_t* hi);
void trace_reset_spdbig();

}  // namespace gpk
