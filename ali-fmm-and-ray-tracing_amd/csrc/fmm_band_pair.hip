// fmm_band_pair.hip — the band-synchronous FMM of fmm_band.hip with TWO workgroups (two CUs)
// per source, so that 128 sources fill the 256 CUs of an MI355X.
//
// Cells are owned by column stripes of 64: member m owns columns with (x >> 6) & 1 == m.  Each
// member keeps the close set, accepted / claimed lists and claim hash of its own cells in LDS and
// evaluates / commits only its own cells; the step is the single-workgroup step with two
// pair barriers (one counter per source, relaxed agent-scope atomics + sc1 polling):
//   P1  local Tmin -> exchange (Tmin, live, err) --X1--  global Tmin; apply the previous step's
//       deferred edge commits
//   P2  accept own cells; own accepted cells next to the partner's columns -> exchange list --X2--
//   P3  claim own neighbours of both members' accepted cells; evaluate them (Jacobi)
//   P4  commit: interior cells directly; EDGE cells (within 2 columns of a stripe boundary, i.e.
//       readable by the partner's 12-cell stencil) are deferred to after the next X1, so the
//       partner never sees a value of this step while it may still be evaluating it.
// X1 carries no bulk data: each member stores its (Tmin, live, err) as four flagged 8-byte words
// (step number in the high half) and polls the partner's, so the exchange is one store and one poll
// round trip.  X2 is a counter barrier: data the partner reads (edge cells' T and status, the rim
// list) is written with sc1 stores and drained (vmcnt 0) before it; the rim list is read with sc1 loads, and
// after X2 one wave invalidates the CU's L1 (agent-scope acquire) so that the claim's status loads
// and the stencil loads are plain loads in one form for every lane.  Results are identical to the
// single-workgroup kernel: the same cells are accepted, claimed and evaluated against the same
// state each step; only which CU does the work differs.
#include <type_traits>
#include "kernels.h"
#include "local_ops.h"
#include "fields.h"
#include "band_common.h"

namespace af {

namespace pair {

#ifndef AF_FBLIST
#define AF_FBLIST 1
#endif
#ifndef AF_PAIR_THREADS
#define AF_PAIR_THREADS 512
#endif
constexpr int kThreads = AF_PAIR_THREADS;
constexpr int kWaves = kThreads / 64;
#ifndef AF_STRIPE_LOG
#define AF_STRIPE_LOG 6
#endif
constexpr int kStripeLog = AF_STRIPE_LOG;
constexpr int kStripe = 1 << kStripeLog;
constexpr int kLcap = 2560, kAcap = 1024, kEcap = 1536, kDcap = 1024;
constexpr int kHashLog = 13;
constexpr int kHash = 1 << kHashLog;
#ifndef AF_CLAIM_U
#define AF_CLAIM_U 4
#endif
constexpr int kClaimU = AF_CLAIM_U;  // claim items per lane per pass
constexpr int kHashItems = 6144;  // claim items (both members' accepted cells x 4) for the LDS hash
constexpr int kStabLds = 64, kPtabLds = 722, kMatLds = 256;

struct Lds {
  double red[kWaves];
  double Lt[kLcap];
  double Vl[kEcap];
  double Dv[kDcap];  // deferred edge commits: value
  double stab[kStabLds * 5];
  double ptab[kPtabLds];
  MatRec mat[kMatLds];
  int Ll[kLcap];
  int Fs[kLcap];
  int Al[kAcap];
  int El[kEcap];
  int Ep[kEcap];
  int Dc[kDcap];  // deferred edge commits: packed cell
  int Ds[kDcap];  // deferred edge commits: new status (1 + slot) or 0 for "T only"
  alignas(16) int H[kHash];
  int Px[kThreads];  // the partner's rim list, first kThreads entries (prefetched after X2)
  double tmin_g;
  int nA, nE, nF, hi, taken, nD, nAx, live_g, err_g, err, nFb;
};

AF_DEV bool mine(int x, int m) { return ((x >> kStripeLog) & 1) == m; }
// within 2 columns of a stripe boundary: the partner's stencils (update() and fouds18_A()) read it
AF_DEV bool edge(int x) {
  const int r = x & (kStripe - 1);
  return r < 2 || r >= kStripe - 2;
}
// next to a stripe boundary: its x-neighbour belongs to the partner
AF_DEV bool rim(int x) {
  const int r = x & (kStripe - 1);
  return r == 0 || r == kStripe - 1;
}
AF_DEV unsigned hslot(int key) { return ((unsigned)key * 2654435761u) >> (32 - kHashLog); }
// probe stride of key (double hashing): odd, so the sequence visits every slot
AF_DEV unsigned hstep(int key) { return (((unsigned)key * 0x85ebca6bu) >> (32 - kHashLog)) | 1u; }

// two-member barrier; false on timeout (the partner never arrived: both members then stop).
// acquire = true: wave 0 invalidates the CU's vector L1 (agent-scope acquire, buffer_inv sc1)
// after the partner's arrival, so that every later plain load of the step sees the partner's
// (and this workgroup's own sc1-stored) edge data from L2
AF_DEV bool pair_barrier(int* ctr, int& gen, Lds* sh, bool acquire = false) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores are complete
  __syncthreads();
  if (threadIdx.x == 0) {
    const int before = __hip_atomic_fetch_add((AF_GLOBAL int*)ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    gen += 2;
    long spins = 0;
    // the second member to arrive learns it from its own add (no poll round trip on the step's
    // critical path); the first polls
    while (before + 1 < gen && gld_sc1(ctr) < gen) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1L << 25)) {  // ~seconds: never reached unless the partner is not resident
        sh->err = 7;
        break;
      }
    }
  }
  if (acquire && threadIdx.x < 64) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __syncthreads();
  return sh->err != 7;
}

template <int MODE, bool LDSMAT, bool PROF>
__global__ __launch_bounds__(kThreads) void fmm_band_pair_kernel(BandParams P) {
  __shared__ Lds sh_;
  Lds* sh = &sh_;
  const int b = blockIdx.x;
  const int src = (b / 16) * 8 + (b % 8), me = (b / 8) & 1, pt = me ^ 1;
  if (src >= P.nsrc) return;  // both members of a pair take this exit together
  BandSrc* B = P.src + src;
  PairX* X = B->px;
  const int tid0 = threadIdx.x;
  const int tid = tid0, lane = tid & 63, wv = tid >> 6;
  const int nz = P.nz, nx = P.nx;
  double* T = B->T;
  int* S = B->S;
  int* own = B->own;
  int* AXm = B->ax[me];
  const int* AXp = B->ax[pt];
  DevModel M = P.M;
  if (LDSMAT) {
    for (int k = tid; k < 5 * M.nstab; k += kThreads) sh->stab[k] = M.stab[k];
    for (int k = tid; k < 361 * M.ncol; k += kThreads) sh->ptab[k] = M.ptab[k];
    for (int k = tid; k < M.nmat; k += kThreads) sh->mat[k] = M.mtab[k];
    M.ptab = sh->ptab;
  }
  // per-member halves of the work arrays (global spill of the LDS lists)
  const long hL = P.capL / 2, hC = P.capC / 2;
  const HList<int, kLcap> L{sh->Ll, B->L0 + me * hL};
  const HList<double, kLcap> Lt{sh->Lt, B->Lt0 + me * hL};
  const HList<int, kLcap> FS{sh->Fs, B->L1 + me * hL};
  const HList<int, kAcap> AL{sh->Al, B->A + me * hL};
  const HList<int, kEcap> EL{sh->El, B->C + me * hC};
  const HList<int, kEcap> EP{sh->Ep, B->Cp + me * hC};
  const HList<double, kEcap> VL{sh->Vl, B->V + me * hC};
  const int capL = (int)hL, capC = (int)hC;
  if (tid == 0) {
    sh->hi = 0;
    sh->nF = 0;
    sh->nD = 0;
    sh->err = 0;
  }
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
        if (mine(x, me)) {
          t = H->ttn[k];
          gst_sc1(T + c, t);
          if (H->cls[k] == 1) gst_sc1(S + c, (int)kKnown);
          else push = true;
        }
      }
      const int s = wave_push(&sh->hi, push, capL, &sh->err);
      if (s >= 0) {
        L.put(s, pk(z, x));
        Lt.put(s, t);
        gst_sc1(S + c, 1 + s);
      }
    }
  } else {
    if (tid == 0 && B->err) sh->err = B->err;
    const int n = B->nl0;
    for (int k0 = wv * 64; k0 < n; k0 += kThreads) {
      const int k = k0 + lane;
      bool push = false;
      int c = 0, z = 0, x = 0;
      if (k < n) {
        c = gld(B->L0 + k);
        z = c / nx;
        x = c - z * nx;
        push = mine(x, me);
      }
      // both members read all of L0 before either rewrites its half (member 0's half starts at
      // L0[0]): stage the own cells first, then rewrite after the barrier below
      const int s = wave_push(&sh->hi, push, capL, &sh->err);
      if (s >= 0) {  // cells staged in the (still unused) free-stack arrays, copied after the barrier
        Lt.put(s, gld(T + c));
        FS.put(s, pk(z, x));
        gst_sc1(S + c, 1 + s);
      }
    }
  }
  int gen = 0;
  // both members have read the hand-over input and written their statuses
  pair_barrier(&X->bar, gen, sh);
  if (MODE == 1) {
    for (int k = tid; k < sh->hi; k += kThreads) L.put(k, FS.get(k));
    __syncthreads();
  }
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
  const GFieldSC1 F{T, S, nz, nx};
  long long steps = 0, myupd = 0;
  // profile (P.prof): thread 0 of member 0; phases [P1+X1, P2+X2, claim, evaluate, fallback, commit],
  // sub [X1 wait, X2 wait, claim dedupe (waited), claim status loads] — BandSrc::ph / sub, same layout as fmm_band.hip
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
    // the thread index is re-read each step (opaque to the compiler), so values derived from it
    // (per-lane list addresses) are recomputed in the step instead of being kept live across the
    // whole loop and spilled to scratch (a memory round trip per reload)
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wv = tid >> 6;
    const int par = (int)(steps & 1);
    const int hi = sh->hi;
    // ---- P1: local Tmin, exchange ----
    double tmin = INFINITY;
    if (hi <= kLcap) {  // (uniform) close set in LDS: plain LDS reads the compiler can batch
      for (int e = tid; e < hi; e += kThreads) tmin = fmin(tmin, Lt.lds(e));
    } else {
      for (int e = tid; e < hi; e += kThreads) tmin = fmin(tmin, Lt.get(e));
    }
    for (int k = tid * 4; k < kHash; k += kThreads * 4) *(int4*)&sh->H[k] = make_int4(0, 0, 0, 0);
    tmin = wave_min(tmin);
    if (lane == 0) sh->red[wv] = tmin;
    __syncthreads();
    const long long tx1 = prof ? wall_clock64() : 0;
    if (tid == 0) {
      double t = sh->red[0];
      for (int w = 1; w < kWaves; w++) t = fmin(t, sh->red[w]);
      sh->nA = 0;
      sh->nAx = 0;
      sh->nE = 0;
      sh->nFb = 0;
      sh->taken = 0;
      // X1: flagged words out, the partner's in.  No drain: nothing this member stored is read by
      // the partner before X2 (which drains); seeing the partner's words means it has finished
      // the previous step (its evaluation loads were consumed before its commit).
      const unsigned long long g = (unsigned long long)(steps + 1) << 32;
      const unsigned long long tb = (unsigned long long)__double_as_longlong(t);
      const int live = hi - sh->nF;
      gst_sc1(&X->x1[me][0], g | (tb & 0xffffffffull));
      gst_sc1(&X->x1[me][1], g | (tb >> 32));
      gst_sc1(&X->x1[me][2], g | (unsigned)live);
      gst_sc1(&X->x1[me][3], g | (unsigned)sh->err);
      unsigned long long w0, w1, w2, w3;
      long spins = 0;
      while (true) {
        w0 = gld_sc1(&X->x1[pt][0]);
        w1 = gld_sc1(&X->x1[pt][1]);
        w2 = gld_sc1(&X->x1[pt][2]);
        w3 = gld_sc1(&X->x1[pt][3]);
        if (((w0 & w1 & w2 & w3) >> 32) == (g >> 32) && ((w0 | w1 | w2 | w3) >> 32) == (g >> 32)) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1L << 25)) {  // ~seconds: never reached unless the partner is not resident
          sh->err = 7;
          break;
        }
      }
      const double tp = __longlong_as_double((long long)((w0 & 0xffffffffull) | (w1 << 32)));
      sh->tmin_g = fmin(t, tp);
      sh->live_g = live + (int)(unsigned)w2;
      sh->err_g = sh->err | (int)(unsigned)w3;
    }
    __syncthreads();
    AF_SUBT(0, tx1)
    const long long tap = prof ? wall_clock64() : 0;
    // apply the previous step's deferred edge commits (the partner finished evaluating it)
    for (int d = tid; d < sh->nD; d += kThreads) {
      const int c = sh->Dc[d];
      const long f = (long)pkz(c) * nx + pkx(c);
      gst_sc1(T + f, sh->Dv[d]);
      if (sh->Ds[d] > 0) gst_sc1(S + f, sh->Ds[d]);
    }
    __syncthreads();
    AF_TICK(0)
    if (sh->live_g <= 0 || sh->err_g || sh->err == 7) break;
    if (tid == 0) sh->nD = 0;
    tmin = sh->tmin_g;
    const double delta = launder_u(R.delta), t0 = launder_u(R.t0);
    double dl = delta;
    if (t0 > 0 && tmin < t0) dl = delta * (tmin / t0);
    const double thr = tmin + dl;
    // ---- P2: accept own cells; rim cells go to the exchange list ----
    int* nax = &sh->nAx;  // reset with nA in P1
    auto accept = [&](auto lds_only) {
      constexpr bool LO = decltype(lds_only)::value;
      for (int e0 = wv * 64; e0 < hi; e0 += kThreads) {
        const int e = e0 + lane;
        const double t = e < hi ? (LO ? Lt.lds(e) : Lt.get(e)) : INFINITY;
        const bool acc = t <= thr;
        const int c = acc ? (LO ? L.lds(e) : L.get(e)) : 0;
        int sa, sf;
        wave_push2(&sh->nA, &sh->nF, acc, capL, &sh->err, sa, sf);
        if (sa >= 0) {
          AL.put(sa, c);
          const long f = (long)pkz(c) * nx + pkx(c);
          if (edge(pkx(c))) gst_sc1(S + f, (int)kKnown);
          else gst(S + f, (int)kKnown);
          if (LO) {
            Lt.put_lds(e, INFINITY);
            FS.put_lds(sf, e);
          } else {
            Lt.put(e, INFINITY);
            FS.put(sf, e);
          }
        }
        const int sx = wave_push(nax, acc && rim(pkx(c)), capL, &sh->err);
        if (sx >= 0) gst_sc1(AXm + sx, c);
      }
    };
    // (uniform) close set and free stack in LDS (slots and free-stack entries are < hi)
    if (hi <= kLcap) accept(std::true_type{});
    else accept(std::false_type{});
    __syncthreads();
    if (tid == 0) gst_sc1(&X->nax[me][par], *nax);
    const long long tx2 = prof ? wall_clock64() : 0;
    if (!pair_barrier(&X->bar, gen, sh, true)) break;  // X2 (+ L1 invalidate)
    AF_SUBT(1, tx2)
    AF_TICK(1)
    const int nA = min(sh->nA, capL);
    // the partner's rim count and the head of its list in ONE round trip (entries past the count
    // are stale and never read), staged in LDS
    const int nAp = gld_sc1(&X->nax[pt][par]);
    sh->Px[tid] = gld_sc1(AXp + tid);
    __syncthreads();
    // ---- P3a: claim own neighbours of own accepted cells and of the partner's rim cells ----
    const int nItems = 4 * (nA + nAp);
    const bool use_hash = nItems <= kHashItems;
    const bool lds_items = nA <= kAcap && nAp <= kThreads;
    const int stamp = (int)steps;
    for (int q0 = wv * 64 * kClaimU; q0 < nItems; q0 += kThreads * kClaimU) {
      int r[kClaimU], s[kClaimU], o[kClaimU];
      const long long tdd = prof ? wall_clock64() : 0;
      // first probe of all 8 items issued back to back (one LDS round trip), collisions after
      unsigned hh[kClaimU];
      int pv[kClaimU];
      if (lds_items) {  // (uniform) both lists in LDS: branch-free item generation
#pragma unroll
        for (int u = 0; u < kClaimU; u++) {
          const int q = q0 + u * 64 + lane;
          const int a = q >> 2;
          const int ac = a < nA ? AL.lds(a) : sh->Px[a - nA < kThreads ? a - nA : 0];
          int c = nb_cell(ac, q & 3, nz, nx);
          if (q >= nItems || (c >= 0 && !mine(pkx(c), me))) c = -1;
          r[u] = c;
          hh[u] = hslot(c);
        }
      } else {
#pragma unroll
        for (int u = 0; u < kClaimU; u++) {
          const int q = q0 + u * 64 + lane;
          int c = -1;
          if (q < nItems) {
            const int a = q >> 2;
            const int ap = a - nA;
            const int ac = a < nA ? AL.get(a) : ap < kThreads ? sh->Px[ap] : gld_sc1(AXp + ap);
            c = nb_cell(ac, q & 3, nz, nx);
            if (c >= 0 && !mine(pkx(c), me)) c = -1;
          }
          r[u] = c;
          hh[u] = hslot(c);
        }
      }
      if (use_hash) {
#pragma unroll
        for (int u = 0; u < kClaimU; u++) pv[u] = r[u] >= 0 ? atomicCAS(&sh->H[hh[u]], 0, r[u] + 1) : 0;
        // collisions: double hashing (odd key-dependent stride: no primary clusters), all 8
        // items in ONE loop whose trip count is the longest probe sequence among them
        unsigned pend = 0;
#pragma unroll
        for (int u = 0; u < kClaimU; u++) {
          if (pv[u] != 0) {
            if (pv[u] == r[u] + 1) r[u] = -1;  // already claimed
            else pend |= 1u << u;
          }
        }
        for (int probe = 1; pend; probe++) {
          if (probe >= kHash) {
            sh->err = 5;
#pragma unroll
            for (int u = 0; u < kClaimU; u++)
              if ((pend >> u) & 1u) r[u] = -1;
            break;
          }
#pragma unroll
          for (int u = 0; u < kClaimU; u++) {
            if ((pend >> u) & 1u) {
              hh[u] = (hh[u] + hstep(r[u])) & (kHash - 1);
              pv[u] = atomicCAS(&sh->H[hh[u]], 0, r[u] + 1);
              if (pv[u] == 0 || pv[u] == r[u] + 1) {
                if (pv[u] != 0) r[u] = -1;
                pend &= ~(1u << u);
              }
            }
          }
        }
      }
      if (prof) __builtin_amdgcn_s_waitcnt(0);
      AF_SUBT(2, tdd)
      const long long tcl = prof ? wall_clock64() : 0;
#pragma unroll
      for (int u = 0; u < kClaimU; u++) {
        const long f = r[u] >= 0 ? (long)pkz(r[u]) * nx + pkx(r[u]) : 0;
        s[u] = r[u] >= 0 ? gld(S + f) : (int)kKnown;  // L1 invalidated at X2
        o[u] = (!use_hash && r[u] >= 0) ? gatomic_max(own + f, stamp) : -1;
      }
      // u-major list order: consecutive entries are neighbours of consecutive accepted cells, so
      // the lanes of an evaluating wave read overlapping stencils (fewer distinct cache lines)
      unsigned long long bm[kClaimU];
      int cnt = 0;
#pragma unroll
      for (int u = 0; u < kClaimU; u++) {
        bm[u] = __ballot(s[u] != kKnown && o[u] < stamp);
        cnt += __popcll(bm[u]);
      }
      AF_SUBT(3, tcl)
      int base = 0;
      if (lane == 0 && cnt) base = atomicAdd(&sh->nE, cnt);
      base = __shfl(base, 0);
      const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
      for (int u = 0; u < kClaimU; u++) {
        if ((bm[u] >> lane) & 1ull) {
          const int pos = base + __popcll(bm[u] & lt);
          if (pos < capC) {
            EL.put(pos, r[u]);
            EP.put(pos, s[u] > 0 ? s[u] - 1 : -1);
          } else {
            sh->err = 2;
          }
        }
        base += __popcll(bm[u]);
      }
    }
    __syncthreads();
    AF_TICK(2)
    const int nE = min(sh->nE, capC);
    // ---- P3b: evaluate (cells whose stencil reaches the partner's columns: sc1 loads) ----
    const bool lds_e = nE <= kEcap;  // (uniform) the claimed list is in LDS
    const double dnx_e = launder_u(R.dnx);
    for (int e = tid; e < nE; e += kThreads) {
      const int r = lds_e ? EL.lds(e) : EL.get(e);
      const int z = pkz(r), x = pkx(r);
      NbFieldT nb;  // stencil loads first, then the material id: one memory round trip
      nb.load(T, nz, nx, z, x);  // L1 invalidated at X2: plain loads see the partner's edge cells
      const CellMat cm = band_mat<LDSMAT>(M, sh->mat, sh->stab, R.mv, z, x);
      const double v = update(nb, M, cm, z, x, dnx_e, nz, nx);
      if (lds_e) VL.put_lds(e, v);
      else VL.put(e, v);
      myupd++;
#if AF_FBLIST
      // no usable stencil: queue the cell for the fouds18_A() pass (the claim hash is free now)
      const unsigned long long fm = __ballot(v == -1.0);
      if (fm) {
        const int fl = __ffsll((long long)fm) - 1;
        int fb = 0;
        if (lane == fl) fb = atomicAdd(&sh->nFb, __popcll(fm));
        fb = __shfl(fb, fl) + __popcll(fm & ((1ull << lane) - 1ull));
        if (v == -1.0 && fb < kHash) sh->H[fb] = e;
      }
#endif
    }
    AF_TICK(3)
    const double dnx_f = launder_u(R.dnx), dnz_f = launder_u(R.dnz);
#if AF_FBLIST
    // fouds18_A() over the compacted list: every fallback cell of the step in parallel lanes (one
    // fouds18_A() latency on the critical path instead of one per evaluation round per wavefront)
    __syncthreads();
    const int nFb = sh->nFb;
    for (int f = tid; f < nFb; f += kThreads) {
      const int e = f < kHash ? sh->H[f] : -1;
      if (e >= 0) {
        const int r = EL.get(e);
        const int z = pkz(r), x = pkx(r);
        const CellMat cm = band_mat<LDSMAT>(M, sh->mat, sh->stab, R.mv, z, x);
        VL.put(e, fouds18<true>(F, M, cm, z, x, dnx_f, dnz_f, nx, nz, mat_slo(M, R.mv, z, x)));
      }
    }
    if (nFb > kHash) {  // list overflow (more fallback cells than hash slots): the rest by scan
      __syncthreads();
      for (int e = tid; e < nE; e += kThreads) {
        if (VL.get(e) == -1.0) {
          const int r = EL.get(e);
          const int z = pkz(r), x = pkx(r);
          const CellMat cm = band_mat<LDSMAT>(M, sh->mat, sh->stab, R.mv, z, x);
          VL.put(e, fouds18<true>(F, M, cm, z, x, dnx_f, dnz_f, nx, nz, mat_slo(M, R.mv, z, x)));
        }
      }
    }
#else
    for (int e = tid; e < nE; e += kThreads) {
      if (VL.get(e) == -1.0) {
        const int r = EL.get(e);
        const int z = pkz(r), x = pkx(r);
        const CellMat cm = band_mat<LDSMAT>(M, sh->mat, sh->stab, R.mv, z, x);
        VL.put(e, fouds18<true>(F, M, cm, z, x, dnx_f, dnz_f, nx, nz, mat_slo(M, R.mv, z, x)));
      }
    }
#endif
    __syncthreads();
    AF_TICK(4)
    // ---- P4: commit own cells; edge cells deferred to after the next X1 ----
    const int nF = sh->nF;
    auto commit = [&](auto lds_only) {
      constexpr bool LO = decltype(lds_only)::value;
      for (int e0 = wv * 64; e0 < nE; e0 += kThreads) {
        const int e = e0 + lane;
        bool fresh = false, defer = false;
        int r = 0;
        double v = 0.0;
        if (e < nE) {
          r = LO ? EL.lds(e) : EL.get(e);
          v = LO ? VL.lds(e) : VL.get(e);
          const int p = LO ? EP.lds(e) : EP.get(e);
          defer = edge(pkx(r));
          if (!defer) gst(T + (long)pkz(r) * nx + pkx(r), v);
          if (p >= 0) {
            if (LO) Lt.put_lds(p, v);
            else Lt.put(p, v);
          } else {
            fresh = true;
          }
        }
        const int k = wave_push(&sh->taken, fresh, 1 << 30, &sh->err);
        int slot = -1;
        if (k >= 0) {
          slot = k < nF ? (LO ? FS.lds(nF - 1 - k) : FS.get(nF - 1 - k)) : hi + (k - nF);
          if (slot >= capL) {
            sh->err = 2;
            slot = -1;
          } else {
            if (LO) {
              L.put_lds(slot, r);
              Lt.put_lds(slot, v);
            } else {
              L.put(slot, r);
              Lt.put(slot, v);
            }
            if (!defer) gst(S + (long)pkz(r) * nx + pkx(r), 1 + slot);
          }
        }
        const int dslot = wave_push(&sh->nD, defer, kDcap, &sh->err);
        if (dslot >= 0) {
          sh->Dc[dslot] = r;
          sh->Dv[dslot] = v;
          sh->Ds[dslot] = slot >= 0 ? 1 + slot : 0;
        }
      }
    };
    // (uniform) claimed lists in LDS and every slot a fresh cell can take below kLcap
    if (nE <= kEcap && hi + nE <= kLcap) commit(std::true_type{});
    else commit(std::false_type{});
    __syncthreads();
    if (tid == 0) {
      const int tk_ = sh->taken;
      sh->nF = max(0, nF - tk_);
      sh->hi = hi + max(0, tk_ - nF);
    }
    if (prof) {
      ls[0] += hi - sh->nF;
      ls[1] += nA;
      ls[2] += nE;
      lmax = max(lmax, (long long)hi);
    }
    steps++;
    __syncthreads();
    AF_TICK(5)
  }
#undef AF_TICK
#undef AF_SUBT
  if (prof) {
    for (int k = 0; k < 6; k++) B->ph[k] += ph[k];
    for (int k = 0; k < 4; k++) B->sub[k] += sub[k];
    for (int k = 0; k < 3; k++) B->lsum[k] += ls[k];
    B->lmax = max(B->lmax, lmax);
  }
  for (int o = 32; o > 0; o >>= 1) myupd += __shfl_xor(myupd, o);
  if (lane == 0 && myupd) atomicAdd((unsigned long long*)&B->nupd, (unsigned long long)myupd);
  if (tid == 0) {
    if (me == 0) B->steps[3] = steps;
    const int e = sh->err ? sh->err : sh->err_g;
    if (e) B->err = e;
  }
}

}  // namespace pair
}  // namespace af

// cooperative launch (all 2*nsrc workgroups resident, one per CU); hipErrorCooperativeLaunchTooLarge
// (or any launch error) tells the caller to use the single-workgroup kernel instead
extern "C" hipError_t af_launch_band_pair(const af::BandParams* P, hipStream_t stream) {
  // (mid => the material table and its fouds18_A() slownesses mslo exist: fouds18<true>)
  const bool lds = P->M.mid && P->M.mslo && P->M.nmat <= af::pair::kMatLds && P->M.nstab <= af::pair::kStabLds &&
                   361 * P->M.ncol <= af::pair::kPtabLds;
  if (!lds) return hipErrorNotSupported;
  const dim3 g(16 * ((P->nsrc + 7) / 8)), b(af::pair::kThreads);
  af::BandParams Pc = *P;
  void* args[] = {&Pc};
  const void* fn = P->mode == 0 ? (P->prof ? (const void*)af::pair::fmm_band_pair_kernel<0, true, true>
                                            : (const void*)af::pair::fmm_band_pair_kernel<0, true, false>)
                                : (P->prof ? (const void*)af::pair::fmm_band_pair_kernel<1, true, true>
                                           : (const void*)af::pair::fmm_band_pair_kernel<1, true, false>);
  return hipLaunchCooperativeKernel(fn, g, b, args, 0, stream);
}
