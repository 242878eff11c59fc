// fmm_band_k.hip — band-synchronous FMM over the main grid with K workgroups ("members", one per
// CU) per source, K = 1, 2, 4, 8 or 16.  Replaces the reference's heap-ordered main
// loop (travel :2055-2102, travel_finer_grid :2775-2817).
//
// Ownership.  The grid is cut into column stripes of W = 2^wlog columns; stripe s belongs to member
// (s mod K).  A member keeps the close set and the accepted / claimed lists of its own cells
// in LDS, and evaluates and commits only its own cells.  Per step (one cross-member exchange):
//   P1  local Tmin over the own close set (LDS); publish the own close RIM cells (next to a stripe
//       boundary) with their T; then X1: every member stores (Tmin, live, err, #rim) as flagged
//       words and reads everybody's -> global Tmin, threshold, termination
//   P2  accept own close cells with T <= thr (-> known, slot freed); bring this step's edge buffer
//       up to date (below)
//   P3  claim own non-known 4-neighbours of own accepted cells and of the neighbour members'
//       accepted rim cells (read from their published lists: T <= thr), each exactly once by the
//       ownership rule (no deduplication structure); cells whose stencil reaches another member's
//       columns go to the end of the list
//   P4  evaluate update() (fallback fouds18_A()) Jacobi-style against the state of the end of the
//       previous step: own cells from T, other members' cells from the previous step's edge buffer
//   P5  commit: T, own slots, and EDGE cells (within 2 columns of a stripe boundary: another
//       member's 12-point / 5x5 stencils read them) also into this step's edge buffer
// Why one exchange is enough: evaluation reads T (unchanged by acceptance) and validity
// (known or close, unchanged by acceptance), so only WHICH cells are evaluated depends on this
// step's acceptance — and another member's acceptance of a rim cell (close, T <= thr) is decided
// by data that member published before X1.  fouds18_A() reads known-ness after acceptance: another member's cell is
// known iff it was known at the end of the previous step, or close with T <= thr (exactly that
// member's accept rule).  Results are identical to the one-workgroup kernel (and to any K): the
// same cells are accepted, claimed and evaluated against the same state every step; only which CU
// does the work differs (tests/test_gpu_parity.py).
//
// Edge buffers E[parity] (after T in the field's allocation; 4 columns per stripe, column-major):
// E[k & 1] holds the state of the end
// of step k, written during step k (a member may still read E[(k - 1) & 1] until every member has
// passed step k's X1).  An edge cell's entry is T, with the sign bit set once the cell is known, so
// the statuses of edge cells never cross CUs.  Keeping E[k & 1] complete: this step's commits and
// acceptances write it directly; last step's commits (close cells whose slot carries the DIRTY
// bit) are copied forward by the accept scan, last step's acceptances by a short list (P0).
//
// Cross-CU data (flags, rim lists, edge buffers) is stored with sc1 stores, drained (vmcnt 0) by
// every wave before the flag, and read with sc1 loads after the flag (MI355X_MICROARCH.md
// "inter-workgroup visibility", Valid forms); once every member has reported the same XCD
// (HW_REG_XCC_ID in its exchange word) the stores are plain and complete in that XCD's L2, where
// the sc1 loads are served (AF_XCD_LOCAL).  Flags and rim lists are double-buffered by parity.
#define CR_LDS_TABLES  // cr_math.h tables in LDS (crm::lds_init at kernel start)
#include <algorithm>
#include <type_traits>
#include "kernels.h"
#include "local_ops.h"
#include "fields.h"
#include "band_common.h"
#include "tile_stream.h"

namespace af {
namespace kb {

// Workgroups per CU (AF_WG_PER_CU): 1 = one 768-thread member per CU with the whole LDS; 2 = two
// 384-thread members per CU (of any sources), each with half the LDS, so that one member's
// barrier waits and memory round trips are covered by the other's work (the host then runs
// twice the members per source, choose_members / af_band_wgs_per_cu).
#ifndef AF_WG_PER_CU
#define AF_WG_PER_CU 1
#endif
// 768 threads: 12 waves, 3 per SIMD (the kernel fits 168 VGPRs): the claim and accept passes
// hide more latency (C4 128 sources: 456 -> 437 ms with 512 -> 768, tools/kbench.py).  Several
// members per CU need workgroups the wave placement can pack: at 3 waves per SIMD two 384-thread
// workgroups (2 + 2 + 1 + 1 waves each) do not fit together (measured: the second wave of
// workgroups waits for the first, tools/micro/residency.hip), three 256-thread ones (one wave per
// SIMD each) do.
#ifndef AF_THREADS
#define AF_THREADS (768 / AF_WG_PER_CU)
#endif
constexpr int kThreads = AF_THREADS;
constexpr int kWaves = kThreads / 64;
// LDS heads of the lists (longer lists spill to the global arrays, HList): sized to the LDS left
// (157 KB of 160), the close set to the C4 peak (3 295 live slots of one member at K = 2): 2560 / 1536
// -> 3328 / 1792 took the C4 band from 416 to 405 ms, the accepted list 1024 -> 1536 (the claim
// then stays in LDS and tile-sorted in the widest steps) to 388 ms; 161 KB of LDS in all
// (two members per CU: half of it each, 77.7 KB)
#if AF_WG_PER_CU == 3
#define AF_LCAP_D 960
#define AF_ECAP_D 512
#define AF_ACAP_D 384
#define AF_HASHLOG_D 11
#define AF_SORTB_D 128
#elif AF_WG_PER_CU == 2
#define AF_LCAP_D 1664
#define AF_ECAP_D 896
#define AF_ACAP_D 768
#define AF_HASHLOG_D 11
#define AF_SORTB_D 256
#else
#define AF_LCAP_D 3328
#define AF_ECAP_D 1792
#define AF_ACAP_D 1536
#define AF_HASHLOG_D 13
#define AF_SORTB_D 512
#endif
#ifndef AF_LCAP
#define AF_LCAP AF_LCAP_D
#endif
#ifndef AF_ECAP
#define AF_ECAP AF_ECAP_D
#endif
#ifndef AF_ACAP
#define AF_ACAP AF_ACAP_D
#endif
constexpr int kLcap = AF_LCAP, kAcap = AF_ACAP, kEcap = AF_ECAP;
constexpr int kBcap = 512 / AF_WG_PER_CU, kDcap = 256 / AF_WG_PER_CU, kRcap = 1024 / AF_WG_PER_CU;
#ifndef AF_X1_SLEEP
#define AF_X1_SLEEP 1
#endif
// claim items per lane and pass (the ownership claim; 1, 4 and 6 measured slower)
#ifndef AF_CLAIM_OWN_U
#define AF_CLAIM_OWN_U 2
#endif
constexpr int kCU = AF_CLAIM_OWN_U;
// the boundary list read in place after the interior one (1) or copied behind it (0)
#ifndef AF_BL_INPLACE
#define AF_BL_INPLACE 1
#endif
#ifndef AF_CLAIM_ADAPT
#define AF_CLAIM_ADAPT 1
#endif
#ifndef AF_FB_ROUND
#define AF_FB_ROUND (128 >> (13 - AF_HASHLOG_D))
#endif
#ifndef AF_DIAG_DBL
#define AF_DIAG_DBL 0
#endif
#ifndef AF_PROF_SPILL
#define AF_PROF_SPILL 0
#endif
#ifndef AF_PROF_CLAIM  // diagnostic: sub[2] = the accepted list's tile sort, sub[3] = the claim's closing drain
#define AF_PROF_CLAIM 0
#endif
#ifndef AF_PROF_FBWAIT
#define AF_PROF_FBWAIT 0
#endif
// diagnostic: sub[2] / sub[3] = evaluation time (from the phase start) of the slowest wave with
// interior cells only / with a boundary cell, summed over the steps with both (sub[1]: their count,
// sub[0]: XCD-local steps, x 100)
#ifndef AF_PROF_EVW
#define AF_PROF_EVW 0
#endif
// diagnostic: sub[2] / sub[3] = (1) the close-set scan / the scan + the drain before the X1
// barrier, from the step's start; (2) P0 / P0 + the accept scan, from the X1 barrier
#ifndef AF_PROF_SEG
#define AF_PROF_SEG 0
#endif
// fallback fouds18_A(): four lanes per cell (1) or one (0)
#ifndef AF_F18_SPLIT
#define AF_F18_SPLIT 1
#endif
// evaluate: boundary cells in the first pass (1) or last (0: measured faster, 416 vs 422 ms)
#ifndef AF_EVAL_BFIRST
#define AF_EVAL_BFIRST 0
#endif
// accepted list ordered by 8x8 tile (counting sort over kSortB buckets) before the claim, when it
// has more than AF_SORT_ACC entries (0: never): the claim's status loads and, through the claim
// order, the evaluation's stencil loads of one wavefront then touch few cache lines
#ifndef AF_SORT_ACC
#define AF_SORT_ACC 256
#endif
// ... and only with at most AF_SORT_KMAX members per source (narrow stripes gain nothing from it)
#ifndef AF_SORT_KMAX
#define AF_SORT_KMAX 8
#endif
#ifndef AF_SORTB
#define AF_SORTB AF_SORTB_D
#endif
#ifndef AF_NB_MIX
#define AF_NB_MIX 2
#endif
constexpr int kSortB = AF_SORTB;
AF_DEV int tile_bucket(int c) { return ((pkz(c) >> 3) & (kSortB / 32 - 1)) << 5 | ((pkx(c) >> 3) & 31); }
#ifndef AF_ACC_U
#define AF_ACC_U 1
#endif
constexpr int kAccU = AF_ACC_U;  // close-set entries per lane per accept pass (2 and 4 measured slower)
// model tables staged in LDS (more materials / stiffness rows: the model arrays are read instead)
#ifndef AF_MATLDS
#define AF_MATLDS (256 / AF_WG_PER_CU)
#endif
#ifndef AF_STABLDS
#define AF_STABLDS 64
#endif
constexpr int kStabLds = AF_STABLDS, kPtabLds = 722, kMatLds = AF_MATLDS;
constexpr int kDirty = (int)0x80000000u;  // close-set slot: committed last step (edge cell)
constexpr int kCell = 0x7fffffff;

// host streaming of final tiles (BandParams::hs): completed tiles staged per step (more wait for
// the flush at the end), own tiles per member with an LDS counter
constexpr int kTdCap = ts::kListCap;
constexpr int kTileMax = ts::kOwnTileMax;
// AF_HS_VEC: 16-byte system-scope stores (1) or 8-byte (0)
#ifndef AF_HS_VEC
#define AF_HS_VEC 1
#endif
#ifndef AF_HS_U
#define AF_HS_U 4  // items per thread and batch of stage_tiles
#endif

// LDS of the fallback's staging windows (kFbRound x 25 doubles)
constexpr int kHashArr = AF_FB_ROUND * 25 * 2;

struct Lds {
  double red[kWaves];
  double Lt[kLcap];  // close set: T of the slot (+inf: free)
  double Vl[kEcap];  // evaluated values
  double stab[kStabLds * 5];
  double ptab[kPtabLds];
  MatRec mat[kMatLds];
  int Ll[kLcap];  // close set: cell of the slot (| kDirty)
  int Fs[kLcap];  // free slots
  int Al[kAcap];  // accepted cells
  int El[kEcap];  // claimed cells (interior first, then the boundary cells of Bl)
  int Ep[kEcap];  // slot of a claimed close cell, -1 for a far cell
  int Bl[kBcap];  // claimed cells whose stencil reaches another member's columns
  int Bp[kBcap];
  int Dc[2][kDcap];  // [step parity]: edge cells accepted in a step (copied forward by the next) ...
  double Dv[2][kDcap];  // ... and their T
  int Rx[kRcap];  // claim items from the neighbour members' accepted rim cells; fallback list
  alignas(16) int H[kHashArr];  // fallback staging windows
#if AF_SORT_ACC
  int As[kAcap];     // the accepted list in tile order
  int Sb[kSortB];    // bucket counts -> offsets
  int Sw[kWaves];    // per-wave bucket sums of the scan
#endif
  // host streaming (BandParams::hs): known-cell counters of the own tiles (two 16-bit counters per
  // word; 0xffff once published), this step's completed tiles (own tile indices)
  unsigned tcnt[kTileMax / 2];
  int Td[2][kTdCap];  // [step parity]: tiles completed in a step (staged, then published later)
  int nTd[2];
  int qpos;      // tiles published (host queue entries written)
  int spos, nst; // tiles staged before this step; tiles staged this step
  int cons;      // tiles the host has taken out of the ring (last read)
  int hsoff;     // streaming given up (ring_space timed out): no more staging or publishing
  double tmin_g;
  unsigned long long nE2;  // claimed-list lengths: interior (low half), boundary (high half)
  int nA, nF, hi, nRx, live_g, err_g, err, nFb;
  int nDb[2];  // [step parity]: lengths of Dc / Dv
  int xl;  // AF_XCD_LOCAL: every member of the source on this member's XCD (set by the exchange)
  int takenb[2], nRb[2];  // [step parity]: fresh close-set slots taken by the commit; rim-list length
  int nrim[2];  // rim-list lengths of the neighbour members (left, right) this step
#if AF_PROF_EVW
  long long evt[kWaves];  // diagnostic: each wave's evaluation end
  int evb[kWaves];        // ... and whether it had cells (1) with a boundary one (2)
#endif
};


// The band kernel's working field Tb (per source, in the arena; its two edge buffers follow it):
// AF_BRICK = 1 stores 4 x 4 bricks of doubles, one 128-byte line each, so the 12-point stencils
// of a wavefront's cells touch fewer lines whatever the direction of the front (modelled on the
// C4 front in the kernel's claim order: 0.87 instead of 1.26 lines per evaluated cell); 0 is
// row-major.  Each member writes the row-major result of its stripes at the end (copy_out_own).
#ifndef AF_BRICK
#define AF_BRICK 1
#endif
struct TbLayout {
  int pitch;  // bricks per brick row (AF_BRICK) or the row pitch
  AF_DEV int at(int z, int x) const {
#if AF_BRICK
    return (((z >> 2) * pitch + (x >> 2)) << 4) | ((z & 3) << 2) | (x & 3);
#else
    return z * pitch + x;
#endif
  }
  // at(z, x) == zpart(z) + xpart(x): the bit fields do not overlap, so a stencil's 12 indices
  // are sums of 5 row parts and 5 column parts
  AF_DEV int zpart(int z) const {
#if AF_BRICK
    return (z >> 2) * (pitch << 4) + ((z & 3) << 2);
#else
    return z * pitch;
#endif
  }
  AF_DEV int xpart(int x) const {
#if AF_BRICK
    return ((x >> 2) << 4) + (x & 3);
#else
    return x;
#endif
  }
};
// stencil indices from the separable row / column parts (1) or per point (0): boundary cells
// (load_nb) and interior cells (load_tb)
#ifndef AF_NB_SEP
#define AF_NB_SEP 1
#endif
#ifndef AF_TB_SEP
#define AF_TB_SEP 0
#endif

// Working field -> row-major result for the stripes member `me` owns (s = me, me + K, ...; stripe
// widths are multiples of 4, so bricks never straddle two owners).  Item = one 4 x 4 brick: one
// contiguous 128-B line read, four 32-B row pieces written; consecutive lanes take consecutive
// bricks of a stripe row, so a wave reads contiguous lines and writes 512-B row segments.
AF_DEV void copy_out_own(double* __restrict__ T, const double* __restrict__ Tb, const TbLayout& L, const KGeom& g,
                         int me, int nz, int nx, int tid) {
  const int nstr = (nx + (1 << g.wlog) - 1) >> g.wlog;
  const int nown = (nstr - me + g.K - 1) / g.K;
  const int qlog = g.wlog - 2;  // bricks per stripe row: 1 << qlog
  const long nq = (long)((nz + 3) >> 2) * nown << qlog;
  const bool vec = AF_BRICK && (nx & 3) == 0;
  for (long q = tid; q < nq; q += kThreads) {
    const int c = (int)(q & ((1 << qlog) - 1));
    const long r = q >> qlog;
    const int zb = (int)(r / nown), js = (int)(r - (long)zb * nown);
    const int x0 = ((me + js * g.K) << g.wlog) + 4 * c, z0 = 4 * zb;
    if (x0 >= nx) continue;
    if (vec && z0 + 4 <= nz) {
      const double2* s = reinterpret_cast<const double2*>(Tb + L.at(z0, x0));
      double2 v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) v[k] = s[k];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        double2* d = reinterpret_cast<double2*>(T + (long)(z0 + i) * nx + x0);
        d[0] = v[2 * i];
        d[1] = v[2 * i + 1];
      }
    } else {
      for (int i = 0; i < 4 && z0 + i < nz; i++)
        for (int k = 0; k < 4 && x0 + k < nx; k++) T[(long)(z0 + i) * nx + x0 + k] = Tb[L.at(z0 + i, x0 + k)];
    }
  }
}

// The band kernel's status array Sb (far -1, known 0, close 1 + close-set slot; per source, in
// the arena): AF_BRICK stores 4 x 8 bricks of int32, one 128-byte line each (claim items — the
// 4-neighbours of tile-ordered accepted cells — then touch 0.17 instead of 0.31 lines per item on
// the C4 front); 0 is row-major.
struct SbLayout {
  int pitch;  // bricks per brick row (AF_BRICK) or the row pitch
  AF_DEV int at(int z, int x) const {
#if AF_BRICK
    return (((z >> 2) * pitch + (x >> 3)) << 5) | ((z & 3) << 3) | (x & 7);
#else
    return z * pitch + x;
#endif
  }
};

// known: 0 (hand-over) or the acceptance stamp -(2 + step); far -1; close 1 + slot
AF_DEV bool sb_known(int s) { return s == 0 || s < -1; }

// 12-point neighbourhood of an interior cell (no other member's columns in reach) from Tb; same
// values and validity as NbFieldT::load (rows past the grid invalid; other out-of-grid positions
// read a clamped address and are never used: update() bounds-checks them)
AF_DEV void load_tb(NbFieldT& nb, const double* Tb, const TbLayout& L, int nz, int nx, int z, int x) {
  const int dz[12] = {0, 0, 0, 0, -2, -1, 1, 2, -1, -1, 1, 1};
  const int dx[12] = {-2, -1, 1, 2, 0, 0, 0, 0, -1, 1, -1, 1};
  nb.iz = z;
  nb.ix = x;
  double t[12];
  if (AF_TB_SEP) {
    int zp[5], xp[5];
#pragma unroll
    for (int r = 0; r < 5; r++) zp[r] = L.zpart(min(max(z + r - 2, 0), nz - 1));
#pragma unroll
    for (int c = 0; c < 5; c++) xp[c] = L.xpart(min(max(x + c - 2, 0), nx - 1));
#pragma unroll
    for (int k = 0; k < 12; k++) t[k] = gld(Tb + (zp[dz[k] + 2] + xp[dx[k] + 2]));
  } else {
#pragma unroll
    for (int k = 0; k < 12; k++) {
      const int zz = min(max(z + dz[k], 0), nz - 1), xx = min(max(x + dx[k], 0), nx - 1);
      t[k] = gld(Tb + L.at(zz, xx));
    }
  }
  unsigned m = 0;
#pragma unroll
  for (int k = 0; k < 12; k++)
    if (z + dz[k] < nz && t[k] == t[k]) m |= 1u << k;
  nb.vm = m;
  nb.t0 = t[0]; nb.t1 = t[1]; nb.t2 = t[2]; nb.t3 = t[3]; nb.t4 = t[4]; nb.t5 = t[5];
  nb.t6 = t[6]; nb.t7 = t[7]; nb.t8 = t[8]; nb.t9 = t[9]; nb.t10 = t[10]; nb.t11 = t[11];
}

// Stencil neighbourhood (NbFieldT) at the state of the end of the previous step: own columns from
// T, other members' columns from the previous step's edge buffer (the known sign dropped).  The
// edge buffers follow T in the field's allocation, so every point is T[idx] with a 32-bit index
// from one base (the loads keep the scalar-base + 32-bit-offset form): 12 independent loads in one
// form (sc1: the edge buffer needs it), issued together.  Out-of-grid positions read a clamped
// index (update() never uses them: it bounds-checks).
AF_DEV void load_nb(NbFieldT& nb, const double* T, const TbLayout& L, int eprv, int total, const KGeom& g, int z,
                    int x) {
  const int dz[12] = {0, 0, 0, 0, -2, -1, 1, 2, -1, -1, 1, 1};
  const int dx[12] = {-2, -1, 1, 2, 0, 0, 0, 0, -1, 1, -1, 1};
  nb.iz = z;
  nb.ix = x;
  int zc[5], cb[5];
  bool ot[5];
#pragma unroll
  for (int r = 0; r < 5; r++) zc[r] = min(max(z + r - 2, 0), g.nz - 1);  // rows z-2 .. z+2 (clamped)
  int idx[12];
  if (AF_NB_SEP) {
    // own points: row part + column part; a column across the stripe boundary (at most the two
    // on one side: stripes are >= 8 wide) is edge-buffer column ecol(x + dx) = e0 + dx, with e0
    // from this cell's stripe s and offset r: s * 4 + r on the left edge, s * 4 + r + 4 - W on the right
    const int W = 1 << g.wlog, r0 = x & (W - 1);
    const int e0 = ((x >> g.wlog) << 2) + r0 + (r0 < 2 ? 0 : 4 - W);
    int zp[5];
#pragma unroll
    for (int r = 0; r < 5; r++) zp[r] = L.zpart(zc[r]);
#pragma unroll
    for (int c = 0; c < 5; c++) {
      ot[c] = g.other(x, c - 2);
      cb[c] = ot[c] ? eprv + (e0 + c - 2) * g.nz : L.xpart(min(max(x + c - 2, 0), g.nx - 1));
    }
#pragma unroll
    for (int k = 0; k < 12; k++) {
      const int r = dz[k] + 2, c = dx[k] + 2;
      idx[k] = ot[c] ? cb[c] + zc[r] : zp[r] + cb[c];  // (in range: no clamp)
    }
  } else {
#pragma unroll
    for (int c = 0; c < 5; c++) {  // columns x-2 .. x+2: own (working field) or edge buffer (column-major)
      ot[c] = g.other(x, c - 2);
      cb[c] = ot[c] ? eprv + g.ecol(x + c - 2) * g.nz : min(max(x + c - 2, 0), g.nx - 1);
    }
#pragma unroll
    for (int k = 0; k < 12; k++) {
      const int r = dz[k] + 2, c = dx[k] + 2;
      const int i = ot[c] ? cb[c] + zc[r] : L.at(zc[r], cb[c]);
      idx[k] = i < 0 ? 0 : i >= total ? total - 1 : i;
    }
  }
  double t[12];
  // 32-bit byte offsets (scalar base + vector offset form) while field + edge buffers stay below
  // 4 GB (2^29 doubles, every C1..C5 grid); larger allocations address with 64-bit pointers
  const bool off32 = total < (1 << 29);  // (uniform)
  if (off32) {
#pragma unroll
    for (int k = 0; k < 12; k++) {
      const double* a = (const double*)((const char*)T + ((unsigned)idx[k] << 3));
      // AF_NB_MIX: own-column points (this member's field: plain loads see its own stores) 1: the
      // cell's own column plain, 2: every own point plain
      if (AF_NB_MIX >= 1 && dx[k] == 0) t[k] = fabs(gld(a));
      else if (AF_NB_MIX == 2) t[k] = fabs(ot[dx[k] + 2] ? gld_sc1(a) : gld(a));
      else t[k] = fabs(gld_sc1(a));
    }
  } else {
#pragma unroll
    for (int k = 0; k < 12; k++) t[k] = fabs(gld_sc1(T + idx[k]));
  }
  unsigned m = 0;
#pragma unroll
  for (int k = 0; k < 12; k++)
    if (z + dz[k] < g.nz && t[k] == t[k]) m |= 1u << k;
  nb.vm = m;
  nb.t0 = t[0]; nb.t1 = t[1]; nb.t2 = t[2]; nb.t3 = t[3]; nb.t4 = t[4]; nb.t5 = t[5];
  nb.t6 = t[6]; nb.t7 = t[7]; nb.t8 = t[8]; nb.t9 = t[9]; nb.t10 = t[10]; nb.t11 = t[11];
}

// fouds18_A() reads a 5x5 neighbourhood with "known" = status 0 after this step's acceptance.  The
// (rare) fallback cells are processed in rounds: all threads stage each cell's neighbourhood into
// LDS — T at the end of the previous step (NaN -> 0 as GField) and known-ness (own cell: status 0;
// another member's: known in the previous edge buffer, or close with T <= thr) — then one lane per
// cell runs fouds18_A() on the staged window (few registers: the accessor is two LDS reads).
constexpr int kFbRound = AF_FB_ROUND;  // cells per staging round (25 doubles each in the claim-hash space)
static_assert(kFbRound * 25 * sizeof(double) <= kHashArr * sizeof(int), "staging windows fit H");
struct Win5 {
  const double* t;  // 25 values, row-major (dz + 2) * 5 + (dx + 2)
  unsigned known;   // bit (dz + 2) * 5 + (dx + 2)
  int iz, ix;
  AF_DEV int st(long z, long x) const { return (known >> ((z - iz + 2) * 5 + (x - ix + 2))) & 1u ? (int)kKnown : -1; }
  AF_DEV double tt(long z, long x) const { return t[(z - iz + 2) * 5 + (x - ix + 2)]; }
};

// fouds18_A() on a staged window, out of line: the fallback runs for a few per cent of the cells,
// and one shared copy keeps its ~30 KB of code out of the step loop's instruction-cache working set
#ifndef AF_F18_OUTLINE
#define AF_F18_OUTLINE 0
#endif
#if AF_F18_OUTLINE
#define AF_F18_ATTR __attribute__((noinline))
#else
#define AF_F18_ATTR __forceinline__
#endif
template <bool PRE_ONLY>
__device__ AF_F18_ATTR double fouds18_w5(const Win5& F, const DevModel& M, const CellMat& cm, int z,
                                                      int x, double dnx, double dnz, int nx, int nz,
                                                      const double* pre) {
  return fouds18<PRE_ONLY>(F, M, cm, z, x, dnx, dnz, nx, nz, pre);
}

// Host streaming.  Tiles are W columns (one stripe) x TR = 2^tr_log rows; member me's own tiles
// are numbered o = tz * nown + js (stripe s = me + js K).  A tile whose cells are all known is
// final.  Tiles completed in step k are staged in step k + 1, right after the X1 drain: their cells
// go to the member's ring of host slots (tile i of the member to slot i mod rslots, row-major with
// row pitch W; system-scope stores, each wave instruction a contiguous piece), and after the next
// drain (every wave's stores complete) their global indices tz * nstr + s are appended to the
// member's host queue.  A slot is reused once the host has taken its tile (its count in cons).
struct TileStream {
  unsigned long long* ring;  // this member's slots (as bits of doubles)
  unsigned long long* hq;    // this member's queue
  const unsigned* cons;      // tiles of this member the host has copied out (host-written)
  int wlog, trlog, nstr, nown, ntiles, K, me, kmagic, nz, nx, rslots;
  AF_DEV int own(int z, int x) const {
    const int s = x >> wlog;
    return (z >> trlog) * nown + ((s * kmagic) >> 16);
  }
  AF_DEV int total(int z, int x) const {  // cells of the tile holding (z, x)
    const int z0 = z & ~((1 << trlog) - 1), x0 = x & ~((1 << wlog) - 1);
    return min(1 << trlog, nz - z0) * min(1 << wlog, nx - x0);
  }
  AF_DEV void origin(int o, int& z0, int& x0) const {
    const int tz = o / nown, js = o - tz * nown;
    z0 = tz << trlog;
    x0 = (me + js * K) << wlog;
  }
  AF_DEV int global(int o) const {
    const int tz = o / nown, js = o - tz * nown;
    return tz * nstr + me + js * K;
  }
};

// before tiles i0 .. i0 + n - 1 of the member are staged: wait until the host has taken the tiles
// that used their slots (one lane; the cached count is re-read only when it falls short)
AF_DEV void ring_space(Lds* sh, const TileStream& ts, int i0, int n) {
  for (long spins = 0; i0 + n - sh->cons > ts.rslots; spins++) {
    sh->cons = (int)__hip_atomic_load(ts.cons, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (i0 + n - sh->cons <= ts.rslots) break;
    __builtin_amdgcn_s_sleep(2);
    if (spins > (1L << 24)) {  // the host stopped taking tiles: this member streams no more
      sh->hsoff = 1;           // (its source's tiles count as missing: the host copies the field
      return;                  // after the launch), the band itself carries on
    }
  }
}

// own cell (z, x) became known: count it; a completed tile joins list b (the step's parity)
AF_DEV void tile_known(Lds* sh, const TileStream& ts, int z, int x, int b) {
  const int o = ts.own(z, x);
  const unsigned sft = (o & 1) * 16;
  const unsigned old = (atomicAdd(&sh->tcnt[o >> 1], 1u << sft) >> sft) & 0xffffu;
  if ((int)old + 1 == ts.total(z, x)) {
    const int p = atomicAdd(&sh->nTd[b], 1);
    if (p < kTdCap) sh->Td[b][p] = o;
  }
}

typedef double d2v __attribute__((ext_vector_type(2)));
// system-scope 16-byte store (host memory): write-through, complete when the wave's vmcnt drains
AF_DEV void st_sys16(unsigned long long* p, double a, double b) {
  const d2v v = {a, b};
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
AF_DEV void st_sys8(unsigned long long* p, double a) {
  __hip_atomic_store(p, (unsigned long long)__double_as_longlong(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// list b's tiles' cells -> their ring slots (tile i0 + k of the member for entry k; every thread;
// loads of AF_HS_U items, then their stores).  An item is one cell (AF_HS_VEC 0) or two adjacent
// cells of a row (1); consecutive lanes take consecutive items of a tile, so one wave instruction
// writes a contiguous piece of the slot
AF_DEV void stage_tiles(const Lds* sh, int n, int b, int i0, const TileStream& ts, const double* Tb,
                        const TbLayout& TL, int tid) {
  constexpr int kV = AF_HS_VEC ? 2 : 1;
  const int clog = ts.wlog + ts.trlog;
  const int ilog = clog - (kV - 1), rlog = ts.wlog - (kV - 1);  // items per tile / row (log2)
  const long total = (long)n << ilog;
  for (long q0 = tid; q0 < total; q0 += (long)AF_HS_U * kThreads) {
    double v0[AF_HS_U], v1[AF_HS_U];
    long d[AF_HS_U];
    int w[AF_HS_U];  // cells of the item inside the grid (0, 1, 2)
#pragma unroll
    for (int u = 0; u < AF_HS_U; u++) {
      const long q = q0 + (long)u * kThreads;
      d[u] = 0;
      w[u] = 0;
      v0[u] = v1[u] = 0.0;
      if (q < total) {
        const int k = (int)(q >> ilog);
        int z0, x0;
        ts.origin(sh->Td[b][k], z0, x0);
        const int r = (int)(q & ((1L << ilog) - 1));
        const int zr = r >> rlog, xr = kV * (r & ((1 << rlog) - 1));
        const int z = z0 + zr, x = x0 + xr;
        if (z < ts.nz && x < ts.nx) {
          w[u] = (kV == 2 && x + 1 < ts.nx) ? 2 : 1;
          v0[u] = gld(Tb + TL.at(z, x));
          if (w[u] == 2) v1[u] = gld(Tb + TL.at(z, x + 1));
          d[u] = ((long)((i0 + k) % ts.rslots) << clog) + (zr << ts.wlog) + xr;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < AF_HS_U; u++) {
      if (w[u] == 2) {
        st_sys16(ts.ring + d[u], v0[u], v1[u]);
      } else if (w[u] == 1) {
        st_sys8(ts.ring + d[u], v0[u]);
      }
    }
  }
}

// after every wave's stores of list b completed (a drain + barrier): wave 0 appends its tiles to
// the host queue, marks them published and empties the list
AF_DEV void publish_tiles(Lds* sh, const TileStream& ts, int b, int lane) {
  const int n = min(sh->nTd[b], kTdCap), q0 = sh->qpos;
  if (lane < n) {
    const int o = sh->Td[b][lane];
    __hip_atomic_store(ts.hq + q0 + lane, ((unsigned long long)(q0 + lane + 1) << 32) | (unsigned)ts.global(o),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    atomicOr(&sh->tcnt[o >> 1], 0xffffu << ((o & 1) * 16));
  }
  if (lane == 0) {
    sh->qpos = q0 + n;
    sh->nTd[b] = 0;
  }
}

// X1 read side (wave 0): lane l polls word l & 3 of member l >> 2 (K <= kMaxK = 16 members, one
// word per lane) until every member's words carry this step's tag, then the wave reduces them:
// global Tmin, live close cells (sum), error (or), and the neighbour members' rim-list lengths.
// false on timeout (a member is not resident)
// XCD-local cross-member data (AF_XCD_LOCAL): once every member of a source has reported the same
// XCD (HW_REG_XCC_ID, carried in its exchange word 2), the members' edge buffers, rim lists
// and exchange words are stored plainly instead of write-through (sc1): the stores complete in the
// XCD's L2, which the readers' sc1 (L1-bypassing) loads are served from, instead of travelling to
// memory and dropping the line from L2.  Placement is read, not assumed: members on different XCDs
// keep the sc1 stores (MI355X_MICROARCH.md "inter-workgroup visibility").
#ifndef AF_XCD_LOCAL
#define AF_XCD_LOCAL 1
#endif
AF_DEV int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}
template <class T>
AF_DEV void xst(T* p, T v, bool loc) {
  if (AF_XCD_LOCAL && loc) gst(p, v);
  else gst_sc1(p, v);
}

AF_DEV bool x1_poll(KX* X, int K, int par, unsigned tag, Lds* sh, int mprev, int mnext) {
  const int lane = threadIdx.x & 63;
  const int nw = 4 * K;
  unsigned long long v = 0;
  long spins = 0;
  while (true) {
    bool ok = true;
    if (lane < nw) {
      v = gld_sc1(&X->x1[lane >> 2][par][lane & 3]);
      ok = (unsigned)(v >> 32) == tag;
    }
    if (__all(ok)) break;
    if (AF_X1_SLEEP) __builtin_amdgcn_s_sleep(AF_X1_SLEEP);
    if (++spins > (1L << 25)) return false;
  }
  const unsigned w = (unsigned)v;
  // words 1..3 of each member into its lane 4q (DPP quad permutes [1,2,3,3], [2,3,3,3], [3,3,3,3])
  const unsigned w1 = (unsigned)dppm_i<0xF9>((int)w), w2 = (unsigned)dppm_i<0xFE>((int)w),
                 w3 = (unsigned)dppm_i<0xFF>((int)w);
  double tmin = INFINITY;
  int live = 0, err = 0;
  if ((lane & 3) == 0 && lane < nw) {
    const int q = lane >> 2;
    tmin = __longlong_as_double((long long)(((unsigned long long)w1 << 32) | w));
    live = (int)(w2 & 0x0fffffffu);
    err = (int)(w3 >> 24);
    if (q == mprev) sh->nrim[0] = (int)(w3 & 0xffffffu);
    if (K > 2 && q == mnext) sh->nrim[1] = (int)(w3 & 0xffffffu);
  }
  // every member's XCD (bits 28..31 of its word 2) equal to this one's
  const bool other_xcd = (lane & 3) == 0 && lane < nw && (int)(w2 >> 28) != xcc_id();
  const bool same = __ballot(other_xcd) == 0;
  tmin = wave_min_full(tmin);
  live = wave_sum_full(live);
  err = wave_or_full(err);
  if (lane == 0) {
    sh->tmin_g = tmin;
    sh->live_g = live;
    sh->err_g = err;
    sh->xl = same ? 1 : 0;
  }
  return true;
}

template <int MODE, bool LDSMAT, bool PROF>
// 3 waves per SIMD (<= 168 VGPRs) in both layouts: 12 waves per CU = one 768-thread or two
// 384-thread members
#ifndef AF_WPE
#define AF_WPE 1
#endif
#ifndef AF_WPE_N
#define AF_WPE_N 3  // waves per SIMD the registers are sized for
#endif
#if AF_WPE
#define AF_WPE_ATTR __attribute__((amdgpu_waves_per_eu(AF_WPE_N)))
#else
#define AF_WPE_ATTR
#endif
__global__ __launch_bounds__(kThreads) AF_WPE_ATTR void fmm_band_k_kernel(BandParams P) {
  __shared__ Lds sh_;
  Lds* sh = &sh_;
  const int K = P.K;
  // block -> (source, member): the K members of a source have equal blockIdx % 8 (one XCD under
  // the observed round-robin placement: a speed preference, never relied on for correctness)
  const int b = blockIdx.x, xq = b & 7, j = b >> 3;
  const int src = (j / K) * 8 + xq, me = j % K;
  if (src >= P.nsrc) return;  // all members of a padding source exit together
  BandSrc* B = P.src + src;
  if (me == 0 && threadIdx.x == 0) B->t_begin = wall_clock64();
  KX* X = B->kx;
  const int tid0 = threadIdx.x;
  const int tid = tid0, lane = tid & 63, wv = tid >> 6;
  const int nz = P.nz, nx = P.nx;
  const KGeom g{K, P.wlog, nz, nx, (65536 + K - 1) / K};
  // the neighbour members (stripes s - 1 and s + 1 of an own stripe s belong to them)
  const int mprev = me == 0 ? K - 1 : me - 1, mnext = me == K - 1 ? 0 : me + 1;
  double* T = B->T;
  double* const Tb = B->Tb;
  const TbLayout TL{P.tb_pitch};
  const SbLayout SL{P.sb_pitch};
  int* const S = B->S;    // row-major status of fmm_exact_kernel's region (mode 1 hand-over only)
  int* const Sb = B->Sb;  // the band's status
  DevModel M = P.M;
  crm::lds_init();
  if (LDSMAT) {
    for (int k = tid; k < 5 * M.nstab; k += kThreads) sh->stab[k] = M.stab[k];
    for (int k = tid; k < 361 * M.ncol; k += kThreads) sh->ptab[k] = M.ptab[k];
    for (int k = tid; k < M.nmat; k += kThreads) sh->mat[k] = M.mtab[k];
    M.ptab = sh->ptab;
  }
  // per-member slices of the global spill arrays of the LDS lists
  const long hL = P.capL / K, hC = P.capC / K;
  const HList<int, kLcap> L{sh->Ll, B->L + me * hL};
  const HList<double, kLcap> Lt{sh->Lt, B->Lt + me * hL};
  const HList<int, kLcap> FS{sh->Fs, B->FS + me * hL};
  const HList<int, kAcap> AL{sh->Al, B->A + me * hL};
  const HList<int, kEcap> EL{sh->El, B->C + me * hC};
  const HList<int, kEcap> EP{sh->Ep, B->Cp + me * hC};
  const HList<double, kEcap> VL{sh->Vl, B->V + me * hC};
  const HList<int, kBcap> BL{sh->Bl, B->Bl + me * hC};
  const HList<int, kBcap> BP{sh->Bp, B->Bp + me * hC};
  // the accepted-edge-cell lists of the two step parities (global spill: half of the slice each)
  const long hD = hC / 2;
  const int capD = (int)hD;
  const HList<int, kRcap> RX{sh->Rx, B->Rx + me * hC};
  const int capL = (int)hL, capC = (int)hC;
  // rim lists [member][parity][capR]; edge buffers [parity][cells] (selected by arithmetic on the
  // step parity: no dynamically indexed private arrays, which would live in scratch)
  int* const rimc = B->rimc;
  double* const rimt = B->rimt;
  // edge buffer of parity p: Tb + tb_cells + p * ecells, compact (KGeom::eidx)
  const int cells = nz * nx, ecells = (int)P.ecells, tbc = (int)P.tb_cells;
  double* const E0 = Tb + tbc;
  // host streaming (mode 0 only)
  const bool hstream = MODE == 0 && P.hs != nullptr;
  TileStream ts{};
  if (hstream) {
    ts.wlog = P.wlog;
    ts.trlog = P.tr_log;
    ts.nstr = (nx + (1 << P.wlog) - 1) >> P.wlog;
    ts.nown = (ts.nstr - me + K - 1) / K;
    ts.ntiles = ts.nown * ((nz + (1 << P.tr_log) - 1) >> P.tr_log);
    ts.K = K;
    ts.me = me;
    ts.kmagic = g.kmagic;
    ts.nz = nz;
    ts.nx = nx;
    const long mid = (long)src * K + me;
    ts.rslots = max(P.rslots, 1);
    ts.ring = reinterpret_cast<unsigned long long*>(P.hs) + (mid * P.rslots << (P.wlog + P.tr_log));
    ts.hq = P.hq + mid * P.qcap;
    ts.cons = P.hcons + mid;
    for (int k = tid; k < kTileMax / 2; k += kThreads) sh->tcnt[k] = 0u;
  }
  if (tid == 0) {
    sh->nTd[0] = sh->nTd[1] = 0;
    sh->qpos = sh->spos = sh->nst = sh->cons = sh->hsoff = 0;
    sh->hi = 0;
    sh->nF = 0;
    sh->nDb[0] = sh->nDb[1] = 0;
    sh->nRb[0] = sh->nRb[1] = 0;
    sh->takenb[0] = sh->takenb[1] = 0;
    sh->xl = 0;
    sh->err = 0;
    sh->nrim[0] = sh->nrim[1] = 0;
    // a list may be staged and not yet published when the next asks for slots: fewer slots than
    // two lists could wait for the host forever (tile_stream.h kRingSlots)
    if (hstream && P.rslots < 2 * kTdCap) sh->err = 11;
  }
#if AF_SORT_ACC
  for (int k = tid; k < kSortB; k += kThreads) sh->Sb[k] = 0;  // (re-zeroed after each sort)
#endif
  __syncthreads();
  // ---------------- hand-over: own cells only ----------------
  if (MODE == 0) {
    const HandoverOut* H = P.ho + src;
    if (tid == 0 && H->err) sh->err = 3;
    const int n = H->n;
    for (int k0 = wv * 64; k0 < n; k0 += kThreads) {
      const int k = k0 + lane;
      bool push = false;
      int c = 0, z = 0, x = 0;
      double t = 0.0;
      if (k < n) {
        c = H->cell[k];
        z = c / nx;
        x = c - z * nx;
        if (g.owner(x) == me) {
          t = H->ttn[k];
          const bool known = H->cls[k] == 1;
          gst(Tb + TL.at(z, x), t);
          if (g.edge(x)) {
            gst_sc1(E0 + g.eidx(z, x), known ? -t : t);
            gst_sc1(E0 + ecells + g.eidx(z, x), known ? -t : t);
          }
          if (known) {
            gst(Sb + SL.at(z, x), (int)kKnown);
            if (hstream) tile_known(sh, ts, z, x, 1);  // as if completed in step -1
          } else {
            push = true;
          }
        }
      }
      const int s = wave_push(&sh->hi, push, capL, &sh->err);
      if (s >= 0) {
        L.put(s, pk(z, x));
        Lt.put(s, t);
        gst(Sb + SL.at(z, x), 1 + s);
      }
    }
  } else {
    // travel_finer_grid(): fmm_exact_kernel wrote T / S of the exact region and its close cells in
    // Lin; the edge buffers get the region's edge cells (T is NaN outside what it touched)
    // (and every member copies its own columns of the region into the working field)
    if (tid == 0 && B->err) sh->err = B->err;
    {
      const int z0 = max(0, B->bbox[0]), z1 = min(nz - 1, B->bbox[1]);
      const int x0 = max(0, B->bbox[2]), x1 = min(nx - 1, B->bbox[3]);
      const int w = x1 - x0 + 1;
      const long nb = (z1 >= z0 && w > 0) ? (long)(z1 - z0 + 1) * w : 0;
      for (long k = tid; k < nb; k += kThreads) {
        const int z = z0 + (int)(k / w), x = x0 + (int)(k % w);
        if (g.owner(x) == me) {
          const long f = (long)z * nx + x;
          const double t = gld(T + f);
          gst(Tb + TL.at(z, x), t);
          const bool kn = gld(S + f) == kKnown;
          if (kn) gst(Sb + SL.at(z, x), (int)kKnown);
          if (g.edge(x)) {
            const double e = kn ? -t : t;
            gst_sc1(E0 + g.eidx(z, x), e);
            gst_sc1(E0 + ecells + g.eidx(z, x), e);
          }
        }
      }
    }
    const int n = B->nl0;
    for (int k0 = wv * 64; k0 < n; k0 += kThreads) {
      const int k = k0 + lane;
      bool push = false;
      int c = 0, z = 0, x = 0;
      if (k < n) {
        c = gld(B->Lin + k);
        z = c / nx;
        x = c - z * nx;
        push = g.owner(x) == me;
      }
      const int s = wave_push(&sh->hi, push, capL, &sh->err);
      if (s >= 0) {
        L.put(s, pk(z, x));
        Lt.put(s, gld(T + c));
        gst(Sb + SL.at(z, x), 1 + s);
      }
    }
  }
  __syncthreads();
  // the close set's high-water mark, carried in a (uniform) register from step to step: the step's
  // end needs no barrier for it (every thread computes the next value from the commit's count)
  int hi_r = __builtin_amdgcn_readfirstlane(sh->hi);
  RunCfg R;
  R.nz = nz;
  R.nx = nx;
  R.dnx = P.dnx;
  R.dnz = P.dnz;
  if (MODE == 0)
    R.mv = MatView{1, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0};
  else
    R.mv = MatView{P.sg, (P.sg - 1) / 2, 0, P.sg, (P.sg - 1) / 2, 0, 1, 0, 0, 0, 1};
  R.delta = launder_u(P.cdelta * P.dnx / P.vmax);
  R.t0 = launder_u(P.r0 * P.dnx / P.vmax);
  R.delta_far = P.cdelta_far * P.dnx / P.vmax;
  R.tfar = P.r_far > 0 && P.cdelta_far > 0 ? P.r_far * P.dnx / P.vmax : 0.0;
  long long steps = 0, myupd = 0;
  // profile (P.prof): thread 0 of member 0; phases [P1 + X1, accept + rim read, claim,
  // evaluate, fallback, commit], sub [X1 wait, rim read, claim dedupe, drain before X1]
  const bool prof = PROF && tid == 0 && me == 0;
  long long ph[6] = {0, 0, 0, 0, 0, 0}, sub[4] = {0, 0, 0, 0}, ls[3] = {0, 0, 0}, lmax = 0;
  long long tk = prof ? wall_clock64() : 0;
#define AF_TICK(k)                 \
  if (prof) {                      \
    long long t_ = wall_clock64(); \
    ph[k] += t_ - tk;              \
    tk = t_;                       \
  }
#define AF_SUBT(k, t0)                   \
  if (prof) sub[k] += wall_clock64() - (t0);
  while (true) {
    // the thread index is re-read each step (opaque to the compiler), so values derived from it are
    // recomputed in the step instead of being kept live across the loop (and spilled)
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wv = tid >> 6;
    const int par = (int)(steps & 1), prv = par ^ 1;
    const int stampA = -2 - (int)steps;  // status of the cells accepted in this step (the claim's ownership rule)
    double* const Epar = E0 + par * ecells;
    const double* const Eprv = E0 + prv * ecells;
    const int eprv = tbc + prv * ecells;  // Eprv as an index from Tb
    const int hi = hi_r;
    // ---- P0h: ring space for the tiles completed last step (staged after the X1 drain) ----
    if (hstream && tid == 0) {
      sh->spos += sh->nst;
      const int nT = min(sh->nTd[prv], kTdCap);
      sh->nst = nT;
      if (nT > 0 && !sh->hsoff) ring_space(sh, ts, sh->spos, nT);
      if (sh->hsoff) sh->nst = sh->nTd[0] = sh->nTd[1] = 0;
    }
    // ---- P1: local Tmin over the close set (LDS); publish every own close RIM cell (cell, T) for
    // the neighbour members, which keep those with T <= thr ----
    double tmin = INFINITY;
    {
      const bool lo = hi <= kLcap;  // (uniform) close set in LDS
      for (int e0 = wv * 64; e0 < hi; e0 += kThreads) {
        const int e = e0 + lane;
        const double t = e < hi ? (lo ? Lt.lds(e) : Lt.get(e)) : INFINITY;
        tmin = fmin(tmin, t);
        const int c = (K > 1 && t < INFINITY) ? ((lo ? L.lds(e) : L.get(e)) & kCell) : 0;
        const bool pub = K > 1 && t < INFINITY && g.rim(pkx(c));
        const int s = wave_push(&sh->nRb[par], pub, P.capR, &sh->err);
        if (s >= 0) {
          xst(rimc + ((long)me * 2 + par) * P.capR + s, c, (bool)sh->xl);
          xst(rimt + ((long)me * 2 + par) * P.capR + s, t, (bool)sh->xl);
        }
      }
    }
#if AF_PROF_SEG == 1
    if (prof) sub[2] += wall_clock64() - tk;
#endif
    tmin = wave_min_full(tmin);
    if (lane == 0) sh->red[wv] = tmin;
    if (tid == 0) {
      sh->nA = 0;
      sh->nE2 = 0;
      sh->nFb = 0;
      sh->takenb[par] = 0;
      sh->nRx = 0;
      sh->nDb[par] = 0;  // (the last step's P0 read nDb[prv])
    }
    // every wave's cross-member stores (this scan's rim list, the last step's edge-buffer and
    // tile-ring stores) complete before the one barrier, after which thread 0 raises the flags
    const long long tdr = prof ? wall_clock64() : 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#if !AF_PROF_FBWAIT && !AF_PROF_SPILL && !AF_PROF_CLAIM && !AF_PROF_SEG
    AF_SUBT(3, tdr)
#endif
#if AF_PROF_SEG == 1
    if (prof) sub[3] += wall_clock64() - tk;
#endif
    tmin = sh->red[0];
    for (int w = 1; w < kWaves; w++) tmin = fmin(tmin, sh->red[w]);
    const double delta = launder_u(R.delta), t0 = launder_u(R.t0);
    if (hstream && !sh->hsoff) {
      // publish the tiles staged last step (their stores have drained: the wait above), then stage
      // the ones completed last step (slots reserved in P0h)
      if (wv == 0 && sh->nTd[par] > 0) publish_tiles(sh, ts, par, lane);
      const int nT = sh->nst;
      if (nT > 0) stage_tiles(sh, nT, prv, sh->spos, ts, Tb, TL, tid);
    }
    const long long tx1 = prof ? wall_clock64() : 0;
    if (K > 1) {
      if (tid == 0) {
        // X1: flagged words (step + 1 in the high half), one store each; the payload arrives with the flag
        const unsigned long long gtag = (unsigned long long)(unsigned)(steps + 1) << 32;
        const unsigned long long tb = (unsigned long long)__double_as_longlong(tmin);
        const bool loc = sh->xl;
        xst(&X->x1[me][par][0], gtag | (tb & 0xffffffffull), loc);
        xst(&X->x1[me][par][1], gtag | (tb >> 32), loc);
        // word 2: this member's XCD (bits 28..31) and live close cells (a front, far below 2^28)
        xst(&X->x1[me][par][2], gtag | ((unsigned)xcc_id() << 28) | ((unsigned)(hi - sh->nF) & 0x0fffffffu), loc);
        xst(&X->x1[me][par][3], gtag | ((unsigned)min(sh->err, 255) << 24) | (unsigned)min(sh->nRb[par], 0xffffff), loc);
      }
      if (wv == 0 && !x1_poll(X, K, par, (unsigned)(steps + 1), sh, mprev, mnext)) {
        if (lane == 0) sh->err = 7;
      }
    } else if (tid == 0) {
      sh->tmin_g = tmin;
      sh->live_g = hi - sh->nF;
      sh->err_g = sh->err;
    }
    if (tid == 0 && steps >= P.max_steps) sh->err = 8;  // a band that never finishes (cannot happen
                                                       // with valid inputs): stop instead of hanging
    __syncthreads();
#if !AF_PROF_EVW
    AF_SUBT(0, tx1)
#endif
    AF_TICK(0)
    if (sh->live_g <= 0 || sh->err_g || sh->err) break;
    // ---- P0: last step's accepted edge cells into this step's edge buffer.  Only now: every member
    // has passed this step's X1, i.e. finished the previous step, which read this buffer.  The
    // list is the last step's parity (this step's acceptance fills the other one: no barrier) ----
    const HList<int, kDcap> DC{sh->Dc[par], B->D + me * hC + par * hD};
    const HList<double, kDcap> DV{sh->Dv[par], B->Dv + me * hC + par * hD};
    if (K > 1) {
      const HList<int, kDcap> DCp{sh->Dc[prv], B->D + me * hC + prv * hD};
      const HList<double, kDcap> DVp{sh->Dv[prv], B->Dv + me * hC + prv * hD};
      const int nD = min(sh->nDb[prv], capD);
      for (int d = tid; d < nD; d += kThreads) {
        const int c = DCp.get(d);
        xst(Epar + g.eidx(pkz(c), pkx(c)), -DVp.get(d), (bool)sh->xl);
      }
    }
#if AF_PROF_SEG == 2
    if (prof) sub[2] += wall_clock64() - tk;
#endif
    tmin = sh->tmin_g;
    double dl = delta;
    if (t0 > 0 && tmin < t0) dl = delta * (tmin / t0);
#ifndef AF_FAR
#define AF_FAR 1
#endif
    if (AF_FAR) {  // wider band far from the source (options cdelta_far / r_far: 0.6 beyond 256 nodes)
      const double tfar = launder_u(R.tfar);
      if (tfar > 0 && tmin > tfar) dl = delta + (launder_u(R.delta_far) - delta) * fmin(1.0, (tmin - tfar) / tfar);
    }
    const double thr = tmin + dl;  // (every thread: no barrier for it)
    // the neighbour members' rim lists: loads issued now, consumed after the accept scan (P3a)
    int rpc = -1;
    double rpt = INFINITY;
    const int nq = K == 1 ? 0 : K == 2 ? 1 : 2;
    const int nr0 = nq > 0 ? min(sh->nrim[0], P.capR) : 0;
    const int nr1 = nq > 1 ? min(sh->nrim[1], P.capR) : 0;
    if (tid < nr0 + nr1) {
      const int side = tid < nr0 ? 0 : 1, e = tid < nr0 ? tid : tid - nr0;
      const int q = side == 0 ? mprev : mnext;
      rpc = gld_sc1(rimc + ((long)q * 2 + par) * P.capR + e);
      rpt = gld_sc1(rimt + ((long)q * 2 + par) * P.capR + e);
    }
    // ---- P2: accept own close cells; copy last step's commits of edge cells forward ----
    // kAccU entries per lane and pass, one LDS atomic pair per wave and pass for the accepted ones
    auto accept = [&](auto lds_only) {
      constexpr bool LO = decltype(lds_only)::value;
      for (int e0 = wv * 64 * kAccU; e0 < hi; e0 += kThreads * kAccU) {
        double t[kAccU];
        int c[kAccU];
        bool acc[kAccU];
        unsigned long long m[kAccU];
        int tot = 0;
#pragma unroll
        for (int u = 0; u < kAccU; u++) {
          const int e = e0 + u * 64 + lane;
          t[u] = e < hi ? (LO ? Lt.lds(e) : Lt.get(e)) : INFINITY;
          const bool live = t[u] < INFINITY;
          acc[u] = t[u] <= thr;
          const int raw = live ? (LO ? L.lds(e) : L.get(e)) : 0;
          c[u] = raw & kCell;
          if (K > 1 && live) {
            const bool ed = g.edge(pkx(c[u]));
            if (raw < 0 || (acc[u] && ed)) {  // dirty (committed last step) or accepted edge cell
              xst(Epar + g.eidx(pkz(c[u]), pkx(c[u])), acc[u] ? -t[u] : t[u], (bool)sh->xl);
              if (raw < 0 && !acc[u]) {
                if (LO) L.put_lds(e, c[u]);
                else L.put(e, c[u]);
              }
            }
            const int d = wave_push(&sh->nDb[par], acc[u] && ed, capD, &sh->err);
            if (d >= 0) {
              DC.put(d, c[u]);
              DV.put(d, t[u]);
            }
          }
          m[u] = __ballot(acc[u]);
          tot += __popcll(m[u]);
        }
        if (tot == 0) continue;
        int ba = 0, bf = 0;
        if (lane == 0) {
          ba = atomicAdd(&sh->nA, tot);
          bf = atomicAdd(&sh->nF, tot);
        }
        ba = bcast(ba, 0);
        bf = bcast(bf, 0);
        const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
        for (int u = 0; u < kAccU; u++) {
          if (acc[u]) {
            const int e = e0 + u * 64 + lane;
            const int off = __popcll(m[u] & lt);
            const int sa = ba + off, sf = bf + off;
            if (sa >= capL || sf >= capL) {
              sh->err = 2;
            } else {
              AL.put(sa, c[u]);
              gst(Sb + SL.at(pkz(c[u]), pkx(c[u])), stampA);
              if (hstream) tile_known(sh, ts, pkz(c[u]), pkx(c[u]), par);
              if (LO) {
                Lt.put_lds(e, INFINITY);
                FS.put_lds(sf, e);
              } else {
                Lt.put(e, INFINITY);
                FS.put(sf, e);
              }
            }
          }
          ba += __popcll(m[u]);
          bf += __popcll(m[u]);
        }
      }
    };
    if (hi <= kLcap) accept(std::true_type{});
    else accept(std::false_type{});
#if AF_PROF_SEG == 2
    if (prof) sub[3] += wall_clock64() - tk;
#endif
    // ---- P3a: the neighbour members' accepted rim cells -> claim items (their cross neighbour) ----
    const long long trr = prof ? wall_clock64() : 0;
    if (K > 1) {
      auto rim_item = [&](int pc, double pt) {  // the cross-boundary neighbour of an accepted rim cell
        int c = -1;
        if (pt <= thr) {
          const int px = pkx(pc), r = px & ((1 << g.wlog) - 1);
          const int cx = r == 0 ? px - 1 : px + 1;
          if (cx >= 0 && cx < nx && g.owner(cx) == me) c = pk(pkz(pc), cx);
        }
        const int s = wave_push(&sh->nRx, c >= 0, capC, &sh->err);
        if (s >= 0) RX.put(s, c);
      };
      rim_item(rpc, rpt);  // the prefetched first kThreads entries
      for (int e0 = kThreads + wv * 64; e0 < nr0 + nr1; e0 += kThreads) {  // the rest (long lists)
        const int e = e0 + lane;
        int pc = -1;
        double pt = INFINITY;
        if (e < nr0 + nr1) {
          const int side = e < nr0 ? 0 : 1, i = e < nr0 ? e : e - nr0;
          const int q = side == 0 ? mprev : mnext;
          pc = gld_sc1(rimc + ((long)q * 2 + par) * P.capR + i);
          pt = gld_sc1(rimt + ((long)q * 2 + par) * P.capR + i);
        }
        rim_item(pc, pt);
      }
    }
    __syncthreads();
#if !AF_PROF_EVW
    AF_SUBT(1, trr)
#endif
    AF_TICK(1)
    const int nA = min(sh->nA, capL), nRx = min(sh->nRx, capC);
    int* alist = sh->Al;
    const long long tso = prof ? wall_clock64() : 0;
#if AF_SORT_ACC
    if (nA > AF_SORT_ACC && nA <= kAcap && K <= AF_SORT_KMAX) {  // (uniform) counting sort of the accepted list by tile
      for (int a = tid; a < nA; a += kThreads) atomicAdd(&sh->Sb[tile_bucket(sh->Al[a])], 1);
      __syncthreads();
      static_assert(kSortB % 64 == 0 && kSortB / 64 <= kWaves, "one bucket per thread of the first waves");
      int cnt = tid < kSortB ? sh->Sb[tid] : 0, wsum;
      const int ex = wave_excl_scan(cnt, wsum);
      if (lane == 0 && wv < kSortB / 64) sh->Sw[wv] = wsum;
      __syncthreads();
      if (tid < kSortB) {
        int base = 0;
        for (int w = 0; w < wv; w++) base += sh->Sw[w];
        sh->Sb[tid] = base + ex;
      }
      __syncthreads();
      for (int a = tid; a < nA; a += kThreads) {
        const int c = sh->Al[a];
        sh->As[atomicAdd(&sh->Sb[tile_bucket(c)], 1)] = c;
      }
      __syncthreads();
      // the buckets zeroed for the next sort (many barriers away)
      for (int k = tid; k < kSortB; k += kThreads) sh->Sb[k] = 0;
      alist = sh->As;
    }
#endif
#if AF_PROF_CLAIM
    AF_SUBT(2, tso)
#endif
    // ---- P3b: claim ----
    const int nItems = 4 * nA + nRx;
    const bool lds_items = nA <= kAcap && nRx <= kRcap;
    // one claimed cell per lane (r >= 0, status s): far or close non-known cells join the interior
    // or the boundary list (one LDS atomic per wave for both)
    auto emit = [&](int rr, int ss) {
      const bool take = rr >= 0 && !sb_known(ss);
      const bool bnd = take && g.edge(pkx(rr));
      const unsigned long long mi = __ballot(take && !bnd), mb = __ballot(bnd);
      if ((mi | mb) == 0) return;
      unsigned long long base2 = 0;
      if (lane == 0)
        base2 = atomicAdd(&sh->nE2, (unsigned long long)__popcll(mi) | ((unsigned long long)__popcll(mb) << 32));
      base2 = bcast64(base2, 0);
      const unsigned long long lt = (1ull << lane) - 1ull;
      const int slot = ss > 0 ? ss - 1 : -1;
      if ((mi >> lane) & 1ull) {
        const int pos = (int)(unsigned)base2 + __popcll(mi & lt);
        if (pos < capC) {
          EL.put(pos, rr);
          EP.put(pos, slot);
        } else {
          sh->err = 2;
        }
      }
      if ((mb >> lane) & 1ull) {
        const int pos = (int)(unsigned)(base2 >> 32) + __popcll(mb & lt);
        if (pos < capC) {
          BL.put(pos, rr);
          BP.put(pos, slot);
        } else {
          sh->err = 2;
        }
      }
    };
    // Claim by ownership: no deduplication structure.  A cell c next to accepted
    // cells is claimed by exactly one item: the own accepted neighbour a = c - dir[d] with the
    // lowest direction d, else (no own accepted neighbour) the neighbour member's rim cell (RX
    // item; a cell has at most one neighbour across a stripe boundary).  "Accepted this step" is
    // the status stamp the accept scan wrote (-(2 + step)), so an item loads c's status and those
    // of c's own neighbours in the directions before its own — all loads of a lane's kCU items
    // issued together: one memory round trip per pass of kThreads * kCU items (the hash claim
    // below waits for LDS atomics and a status load in every pass of kThreads items).
    {
      // stripe crossings instead of owner(): with K > 1 a column next to one's own belongs to
      // another member exactly when it lies across a stripe boundary
      const int W1 = (1 << g.wlog) - 1;
      const bool one = K == 1;
      // kCU items per lane and pass; one (AF_CLAIM_ADAPT) when one pass of one item per thread
      // holds them all: a second item's instructions would issue for nothing (16 sources: 117.9 ->
      // 115.6 ms; a one-item last pass after full ones measured slower, profiles/r6x/kab_claim_adapt*)
      auto claim_pass = [&](auto ucount, int qa, int qb) {
        constexpr int kU = decltype(ucount)::value;
        for (int q0 = qa; q0 < qb; q0 += kThreads * kU) {
          int r[kU], s[kU], pn[kU][4], si[kU];
          unsigned pm[kU];
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const int q = q0 + u * kThreads + tid;
            int c = -1, dd = 4;
            if (q < nItems) {
              if (q < 4 * nA) {
                dd = q & 3;
                const int ac = lds_items ? alist[q >> 2] : AL.get(q >> 2);
                const int z = pkz(ac) + (dd == 2 ? -1 : dd == 3 ? 1 : 0);
                const int x = pkx(ac) + (dd == 0 ? -1 : dd == 1 ? 1 : 0);
                const int xa = pkx(ac) & W1;
                // in the grid, and own (claimed by its owner from my rim list otherwise)
                const bool ok = z >= 0 && z < nz && x >= 0 && x < nx &&
                                (one || !((dd == 0 && xa == 0) || (dd == 1 && xa == W1)));
                c = ok ? pk(z, x) : -1;
              } else {
                c = lds_items ? RX.lds(q - 4 * nA) : RX.get(q - 4 * nA);
              }
            }
            r[u] = c;
            unsigned m = 0;
            int idx = 0;
            {
              const int cc = max(c, 0), z = pkz(cc), x = pkx(cc), xr = x & W1;
              // a' = c - dir[d']: (z, x + 1), (z, x - 1), (z + 1, x), (z - 1, x); own iff not across
              m = (dd > 0 && x + 1 < nx && (one || xr != W1) ? 1u : 0u) | (dd > 1 && x > 0 && (one || xr != 0) ? 2u : 0u) |
                  (dd > 2 && z + 1 < nz ? 4u : 0u) | (dd > 3 && z > 0 ? 8u : 0u);
              m = c >= 0 ? m : 0u;
              idx = SL.at(z, x);
            }
            pm[u] = m;
            si[u] = idx;
          }
          // the neighbours' status indices from c's: within the 4 x 8 brick +-1 / +-8, else the
          // neighbour brick (x: +-25, z: +-(32 pitch - 24))
          const int zstep = 32 * SL.pitch - 24;
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const int c = max(r[u], 0), xi = pkx(c) & 7, zi = pkz(c) & 3, i0 = si[u];
  #if AF_BRICK
            s[u] = r[u] >= 0 ? gld(Sb + i0) : (int)kKnown;
            pn[u][0] = (pm[u] & 1u) ? gld(Sb + i0 + (xi != 7 ? 1 : 25)) : 0;
            pn[u][1] = (pm[u] & 2u) ? gld(Sb + i0 - (xi != 0 ? 1 : 25)) : 0;
            pn[u][2] = (pm[u] & 4u) ? gld(Sb + i0 + (zi != 3 ? 8 : zstep)) : 0;
            pn[u][3] = (pm[u] & 8u) ? gld(Sb + i0 - (zi != 0 ? 8 : zstep)) : 0;
  #else
            s[u] = r[u] >= 0 ? gld(Sb + i0) : (int)kKnown;
            const int z = pkz(c), x = pkx(c);
            pn[u][0] = (pm[u] & 1u) ? gld(Sb + SL.at(z, x + 1)) : 0;
            pn[u][1] = (pm[u] & 2u) ? gld(Sb + SL.at(z, x - 1)) : 0;
            pn[u][2] = (pm[u] & 4u) ? gld(Sb + SL.at(z + 1, x)) : 0;
            pn[u][3] = (pm[u] & 8u) ? gld(Sb + SL.at(z - 1, x)) : 0;
  #endif
          }
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const bool mine = pn[u][0] != stampA && pn[u][1] != stampA && pn[u][2] != stampA && pn[u][3] != stampA;
            emit(mine && !sb_known(s[u]) ? r[u] : -1, s[u]);
          }
        }
      };
      if (AF_CLAIM_ADAPT && nItems <= kThreads) claim_pass(std::integral_constant<int, 1>{}, 0, nItems);
      else claim_pass(std::integral_constant<int, kCU>{}, 0, nItems);
    }
    // this step's edge-buffer stores (accept scan, P0) precede this step's commits to the same
    // addresses (a wave that issued no load since has not waited for them yet)
    const long long tcw = prof ? wall_clock64() : 0;
#ifndef AF_DRAIN_LATE
#define AF_DRAIN_LATE 0
#endif
    // (AF_DRAIN_LATE: the same wait placed before the commit's barrier instead, where the stores
    // have long completed)
    if (K > 1 && !AF_DRAIN_LATE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#if AF_PROF_CLAIM
    AF_SUBT(3, tcw)
#endif
    const int nEi = min((int)(unsigned)sh->nE2, capC);
    const int nEb = min((int)(unsigned)(sh->nE2 >> 32), capC - nEi);
    if (!AF_BL_INPLACE && nEb > 0) {  // boundary cells after the interior ones
      for (int j2 = tid; j2 < nEb; j2 += kThreads) {
        EL.put(nEi + j2, BL.get(j2));
        EP.put(nEi + j2, BP.get(j2));
      }
      __syncthreads();
    }
    AF_TICK(2)
#if AF_PROF_EVW
    const long long tev0 = PROF ? wall_clock64() : 0;
#endif
    const int nE = nEi + nEb;
    // the claimed cells as one list: interior (EL / EP), then boundary (BL / BP), read in place
    // (AF_BL_INPLACE) or from EL / EP after the copy above; VL and the fallback list index it
    auto cellE = [&](int e, auto lds_only) {
      constexpr bool LO = decltype(lds_only)::value;
      if (AF_BL_INPLACE && e >= nEi) return LO ? BL.lds(e - nEi) : BL.get(e - nEi);
      return LO ? EL.lds(e) : EL.get(e);
    };
    auto slotE = [&](int e, auto lds_only) {
      constexpr bool LO = decltype(lds_only)::value;
      if (AF_BL_INPLACE && e >= nEi) return LO ? BP.lds(e - nEi) : BP.get(e - nEi);
      return LO ? EP.lds(e) : EP.get(e);
    };
    // ---- P4: evaluate ----
    const bool lds_e = nE <= kEcap && (!AF_BL_INPLACE || nEb <= kBcap);  // (uniform) every list in LDS
    const double dnx_e = launder_u(R.dnx);
    auto eval_done = [&](int e, double v) {
      if (lds_e) VL.put_lds(e, v);
      else VL.put(e, v);
      myupd++;
      // no usable stencil: queue the cell for the fouds18_A() pass (Rx is free after the claim)
      const unsigned long long fm = __ballot(v == -1.0);
      if (fm) {
        const int fl = __ffsll((long long)fm) - 1;
        int fb = 0;
        if (lane == fl) fb = atomicAdd(&sh->nFb, __popcll(fm));
        fb = bcast(fb, fl) + __popcll(fm & ((1ull << lane) - 1ull));
        if (v == -1.0 && fb < kRcap) sh->Rx[fb] = e;
      }
    };
    // stencil loads first, then the material id: one memory round trip per cell.  Pass order
    // (AF_EVAL_BFIRST): the boundary cells (the list's tail; their edge-buffer lines come from
    // further away) go to the first pass's lanes, so their latency overlaps the interior passes
    // instead of trailing the phase.  Every wave whose cells are all interior loads T only.
    for (int j = tid; j < nE; j += kThreads) {
      const int e = AF_EVAL_BFIRST ? (j < nEb ? nEi + j : j - nEb) : j;
      const bool interior = AF_EVAL_BFIRST ? j - lane >= nEb : e - lane + 64 <= nEi;  // (wave-uniform)
      const int r = lds_e ? cellE(e, std::true_type{}) : cellE(e, std::false_type{});
      const int z = pkz(r), x = pkx(r);
      NbFieldT nb;
      if (interior) load_tb(nb, Tb, TL, nz, nx, z, x);
      else load_nb(nb, Tb, TL, eprv, tbc + 2 * ecells, g, z, x);
      const CellMat cm = band_mat<LDSMAT, MODE == 0>(M, sh->mat, sh->stab, R.mv, z, x);
#if AF_DIAG_DBL  // diagnostic: a second, opaque update() per cell (its marginal cost), same results
      NbFieldT nb2 = nb;
      double d0 = nb.t0;
      asm volatile("" : "+v"(d0));
      nb2.t0 = d0;
      const double v2 = update(nb2, M, cm, z, x, dnx_e, nz, nx);
      eval_done(e, update(nb, M, cm, z, x, dnx_e, nz, nx) + 0.0 * v2);
#else
      eval_done(e, update(nb, M, cm, z, x, dnx_e, nz, nx));
#endif
    }
    AF_TICK(3)
#if AF_PROF_EVW
    if (PROF && me == 0 && lane == 0) {
      sh->evt[wv] = wall_clock64();
      sh->evb[wv] = wv * 64 >= nE ? 0 : (wv * 64 + 63 >= nEi ? 2 : 1);
    }
#endif
    // ---- P4b: fouds18_A() over the compacted fallback list, in staged rounds ----
    const long long tfw = prof ? wall_clock64() : 0;
    __syncthreads();
#if AF_PROF_EVW
    if (prof) {
      long long ti = 0, tb = 0;
      for (int w = 0; w < kWaves; w++) {
        if (sh->evb[w] == 1) ti = max(ti, sh->evt[w] - tev0);
        if (sh->evb[w] == 2) tb = max(tb, sh->evt[w] - tev0);
      }
      if (ti > 0 && tb > 0) {  // steps with both kinds of wave
        sub[2] += ti;
        sub[3] += tb;
        sub[1] += 100;
      }
      sub[0] += sh->xl ? 100 : 0;    // (kbench: fraction of steps with XCD-local exchange)
    }
#endif
#if AF_PROF_FBWAIT  // diagnostic: sub[3] = the wait for the other waves' evaluation
    AF_SUBT(3, tfw)
#endif
    {
      const int nFb = sh->nFb;
      const double thr_f = thr;
      double* const win = reinterpret_cast<double*>(sh->H);  // kFbRound x 25 doubles
      unsigned* const wmask = reinterpret_cast<unsigned*>(sh->Al);
      const int nlist = min(nFb, kRcap);
      // cells past the list capacity (more fallback cells than list slots) are found by a scan
      const int nscan = nFb > kRcap ? nE : 0;
      for (int r0 = 0; r0 < nlist + nscan; r0 += kFbRound) {
        const int nr = min(kFbRound, nlist + nscan - r0);
        if (tid < nr) wmask[tid] = 0u;
        __syncthreads();
        for (int i = tid; i < nr * 25; i += kThreads) {
          const int q = r0 + i / 25, o = i % 25;
          const int e = q < nlist ? sh->Rx[q] : q - nlist;
          if (q >= nlist && VL.get(e) != -1.0) continue;  // scan part: fallback cells only
          const int c = cellE(e, std::false_type{});
          const int zz = pkz(c) + o / 5 - 2, xx = pkx(c) + o % 5 - 2;
          double t = 0.0;
          bool kn = false;
          if (zz >= 0 && zz < nz && xx >= 0 && xx < nx) {
            const long f = (long)zz * nx + xx;
            if (g.owner(xx) == me) {
              t = far0(gld(Tb + TL.at(zz, xx)));
              kn = sb_known(gld(Sb + SL.at(zz, xx)));
            } else {  // known at the end of the last step (sign), or accepted now (close, T <= thr)
              const double ev = gld_sc1(Eprv + g.eidx(zz, xx));
              t = far0(fabs(ev));
              kn = ev == ev && (signbit(ev) || ev <= thr_f);
            }
          }
          win[i] = t;
          if (kn) atomicOr(&wmask[i / 25], 1u << o);
        }
        __syncthreads();
        if (AF_F18_SPLIT) {
          // four lanes per cell, one candidate of each stencil family per lane (fouds18_part)
          static_assert(4 * kFbRound <= kThreads, "four lanes per fallback cell");
          if (tid < 4 * nr) {
            const int ci = tid >> 2, part = tid & 3;
            const int q = r0 + ci;
            const int e = q < nlist ? sh->Rx[q] : q - nlist;
            if (q < nlist || VL.get(e) == -1.0) {  // (the same for the cell's four lanes)
              const int c = cellE(e, std::false_type{});
              const int z = pkz(c), x = pkx(c);
              const Win5 F{win + 25 * ci, wmask[ci], z, x};
              const CellMat cm = band_mat<LDSMAT, MODE == 0>(M, sh->mat, sh->stab, R.mv, z, x);
              const double dnx_f = launder_u(R.dnx), dnz_f = launder_u(R.dnz);
              F18Part fp = fouds18_part<LDSMAT>(F, M, cm, z, x, dnx_f, dnz_f, nx, nz, mat_slo(M, R.mv, z, x), part);
#pragma unroll
              for (int o = 1; o <= 2; o <<= 1) {
                F18Part ot;
#pragma unroll
                for (int k = 0; k < 4; k++) ot.m[k] = __shfl_xor(fp.m[k], o);
                fp = f18_min(fp, ot);
              }
              if (part == 0) VL.put(e, fouds18_combine(fp, F.tt(z, x)));
            }
          }
        } else if (tid < nr) {
          const int q = r0 + tid;
          const int e = q < nlist ? sh->Rx[q] : q - nlist;
          if (q < nlist || VL.get(e) == -1.0) {
            const int c = cellE(e, std::false_type{});
            const int z = pkz(c), x = pkx(c);
            const Win5 F{win + 25 * tid, wmask[tid], z, x};
            const CellMat cm = band_mat<LDSMAT, MODE == 0>(M, sh->mat, sh->stab, R.mv, z, x);
            const double dnx_f = launder_u(R.dnx), dnz_f = launder_u(R.dnz);
            double v;
            v = fouds18_w5<LDSMAT>(F, M, cm, z, x, dnx_f, dnz_f, nx, nz, mat_slo(M, R.mv, z, x));
            VL.put(e, v);
          }
        }
        __syncthreads();
      }
    }
    // (no barrier here: the one before the fallback rounds, or the last round's, already separates
    // every evaluation and fallback write from the commit)
    if (K > 1 && AF_DRAIN_LATE) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    AF_TICK(4)
    // ---- P5: commit own cells; edge cells also into this step's edge buffer (slot marked DIRTY:
    // the next step's accept scan copies them forward) ----
    const int nF = sh->nF;
    auto commit = [&](auto lds_only) {
      constexpr bool LO = decltype(lds_only)::value;
      for (int e0 = wv * 64; e0 < nE; e0 += kThreads) {
        const int e = e0 + lane;
        bool fresh = false, ed = false;
        int r = 0;
        double v = 0.0;
        if (e < nE) {
          r = cellE(e, lds_only);
          v = LO ? VL.lds(e) : VL.get(e);
          const int p = slotE(e, lds_only);
          gst(Tb + TL.at(pkz(r), pkx(r)), v);
          ed = g.edge(pkx(r));
          if (ed) xst(Epar + g.eidx(pkz(r), pkx(r)), v, (bool)sh->xl);
          if (p >= 0) {
            if (LO) {
              Lt.put_lds(p, v);
              if (ed) L.put_lds(p, r | kDirty);
            } else {
              Lt.put(p, v);
              if (ed) L.put(p, r | kDirty);
            }
          } else {
            fresh = true;
          }
        }
        const int k = wave_push(&sh->takenb[par], fresh, 1 << 30, &sh->err);
        if (k >= 0) {
          const int slot = k < nF ? (LO ? FS.lds(nF - 1 - k) : FS.get(nF - 1 - k)) : hi + (k - nF);
          if (slot >= capL) {
            sh->err = 2;
          } else {
            if (LO) {
              L.put_lds(slot, ed ? (r | kDirty) : r);
              Lt.put_lds(slot, v);
            } else {
              L.put(slot, ed ? (r | kDirty) : r);
              Lt.put(slot, v);
            }
            gst(Sb + SL.at(pkz(r), pkx(r)), 1 + slot);
          }
        }
      }
    };
    if (nE <= kEcap && (!AF_BL_INPLACE || nEb <= kBcap) && hi + nE <= kLcap) commit(std::true_type{});
    else commit(std::false_type{});
    __syncthreads();
    // No barrier at the step's end: the next step's first reads of what this end writes are behind
    // its P1 barrier (nF: X1 by thread 0 itself, the accept after it), the step's hi is in a
    // register, and the per-step counters are double-buffered by step parity (a slow wave may still
    // read takenb[par] here while a fast one resets takenb[par ^ 1] in the next P1)
    const int tk_ = sh->takenb[par];
    hi_r = __builtin_amdgcn_readfirstlane(hi + max(0, tk_ - nF));
    if (tid == 0) {
      sh->nF = max(0, nF - tk_);
      sh->nRb[par] = 0;  // the rim list of step + 2
    }
    if (prof) {
      ls[0] += hi - sh->nF;
      ls[1] += nA;
      ls[2] += nE;
      lmax = max(lmax, (long long)hi);
#if AF_PROF_SPILL  // diagnostic: sub[3] counts the steps whose lists outgrew their LDS heads
      sub[3] += (sh->nA > kAcap ? 1 : 0) + (nE > kEcap ? 1000 : 0) + (hi > kLcap ? 1000000 : 0) +
                0LL;
#endif
    }
    steps++;
    AF_TICK(5)
  }
#undef AF_TICK
#undef AF_SUBT
  // the row-major result: each member writes its own stripes' cells as soon as its source is
  // done, so the copy-out of early sources overlaps the band of the late ones
  __syncthreads();
  copy_out_own(T, Tb, TL, g, me, nz, nx, tid);
  // host streaming: every own tile not yet published (incomplete: cells never reached; past a
  // step's list; or staged in the last steps), in windows of kTdCap tiles, each published once
  // its stores have drained
  if (hstream && !sh->hsoff) {
    // the last step's staged list: its stores drained (every wave), then published
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wv == 0 && sh->nst > 0) publish_tiles(sh, ts, (int)(steps & 1) ^ 1, lane);
    if (tid == 0) {
      sh->spos += sh->nst;
      sh->nst = 0;
    }
    for (int base = 0; base < ts.ntiles; base += kTdCap) {
      if (tid == 0) sh->nTd[0] = 0;
      __syncthreads();
      if (tid < kTdCap && base + tid < ts.ntiles) {
        const int o = base + tid;
        if (((sh->tcnt[o >> 1] >> ((o & 1) * 16)) & 0xffffu) != 0xffffu) sh->Td[0][atomicAdd(&sh->nTd[0], 1)] = o;
      }
      __syncthreads();
      const int nT = sh->nTd[0];
      if (nT > 0) {
        if (tid == 0) ring_space(sh, ts, sh->spos, nT);
        __syncthreads();
        if (sh->hsoff) break;  // (uniform: read after the barrier)
        stage_tiles(sh, nT, 0, sh->spos, ts, Tb, TL, tid);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (wv == 0) publish_tiles(sh, ts, 0, lane);
        if (tid == 0) sh->spos += nT;
      }
      __syncthreads();
    }
  }
  if (prof) {
    for (int k = 0; k < 6; k++) B->ph[k] += ph[k];
    for (int k = 0; k < 4; k++) B->sub[k] += sub[k];
    for (int k = 0; k < 3; k++) B->lsum[k] += ls[k];
    B->lmax = max(B->lmax, lmax);
  }
  for (int o = 32; o > 0; o >>= 1) myupd += __shfl_xor(myupd, o);
  if (lane == 0 && myupd) atomicAdd((unsigned long long*)&B->nupd, (unsigned long long)myupd);
  if (tid == 0) {
    if (me == 0) {
      B->steps[3] = steps;
      B->t_end = wall_clock64();
    }
    const int e = sh->err ? sh->err : sh->err_g;
    if (e) atomicMax(&B->err, e);
  }
}

}  // namespace kb
}  // namespace af

// band-kernel workgroups one CU holds at once (the host sizes K so that every member is resident)
extern "C" int af_band_wgs_per_cu() { return AF_WG_PER_CU; }

extern "C" int af_band_tb_pitch(int nx) { return AF_BRICK ? (nx + 3) / 4 : nx; }
extern "C" int af_band_sb_pitch(int nx) { return AF_BRICK ? (nx + 7) / 8 : nx; }
extern "C" long af_band_sb_cells(int nz, int nx) {
  return AF_BRICK ? 32L * ((nz + 3) / 4) * ((nx + 7) / 8) : (long)nz * nx;
}
extern "C" long af_band_tb_cells(int nz, int nx) {
  return AF_BRICK ? 16L * ((nz + 3) / 4) * ((nx + 3) / 4) : (long)nz * nx;
}

// nsrc (padded to a multiple of 8) x K workgroups, AF_WG_PER_CU per CU, all resident
extern "C" hipError_t af_launch_band_k(const af::BandParams* P, hipStream_t stream) {
  const bool lds = P->M.mid && P->M.mslo && P->M.nmat <= af::kb::kMatLds && P->M.nstab <= af::kb::kStabLds &&
                   361 * P->M.ncol <= af::kb::kPtabLds;
  const dim3 g(8 * ((P->nsrc + 7) / 8) * P->K), b(af::kb::kThreads);
  af::BandParams Pc = *P;
  void* args[] = {&Pc};
  const void* fn;
  if (P->mode == 0) {
    fn = lds ? (P->prof ? (const void*)af::kb::fmm_band_k_kernel<0, true, true>
                        : (const void*)af::kb::fmm_band_k_kernel<0, true, false>)
             : (P->prof ? (const void*)af::kb::fmm_band_k_kernel<0, false, true>
                        : (const void*)af::kb::fmm_band_k_kernel<0, false, false>);
  } else {
    fn = lds ? (P->prof ? (const void*)af::kb::fmm_band_k_kernel<1, true, true>
                        : (const void*)af::kb::fmm_band_k_kernel<1, true, false>)
             : (P->prof ? (const void*)af::kb::fmm_band_k_kernel<1, false, true>
                        : (const void*)af::kb::fmm_band_k_kernel<1, false, false>);
  }
  if (P->coop) return hipLaunchCooperativeKernel(fn, g, b, args, 0, stream);
  // Plain launch: the members of a source wait for each other every step, so every workgroup must
  // be resident at once — checked here against the occupancy of this kernel (the grid is sized to
  // it: K from af_band_wgs_per_cu and the CU count).  A cooperative launch checks the same and
  // gang-schedules on a dedicated queue; the plain launch avoids that queue, whose teardown at
  // process exit crashed every rocprofv3-traced run (the profiler's queue interception is gone by
  // then).  A member that still never sees its peers stops at the X1 spin limit (error 7).
  int dev = 0, ncu = 0, per_cu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, af::kb::kThreads, 0);
  if (e != hipSuccess) return e;
  if ((long)per_cu * ncu < (long)g.x) return hipErrorCooperativeLaunchTooLarge;
  return hipLaunchKernel(fn, g, b, args, 0, stream);
}
