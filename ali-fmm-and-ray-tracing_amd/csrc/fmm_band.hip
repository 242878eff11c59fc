// fmm_band.hip — band-synchronous ("Delta-stepping") FMM on gfx950.
//
// Replaces the reference's heap-ordered main loop (travel :2055-2102, travel_finer_grid
// :2775-2817).  One persistent 512-thread workgroup per source; all synchronisation is
// workgroup-local (s_barrier), so sources never wait on each other.  Per step:
//   1  Tmin over the close set — LDS only: the close set is an LDS slot array of (cell, T);
//      a close cell keeps its slot until accepted (nsts = 1 + slot, the reference's "heap index
//      > 0" convention), freed slots go to a free stack
//   2  accept every close cell with T <= Tmin + delta(Tmin) -> known (nsts 0)
//   3a claim: the neighbours of the accepted cells are deduplicated in an LDS hash set; each
//      distinct neighbour's nsts is read once (known: dropped; close: its slot; far: fresh)
//   3b evaluate the reference's update() (fallback fouds18_A()) for every claimed neighbour,
//      Jacobi-style against the post-acceptance state (far cells hold NaN: fields.h NbFieldT)
//   4  commit: T <- new value; far cells take a free slot (nsts = 1 + slot), close cells update
//      their slot's T
// Lists live in LDS and spill to global arrays of the same index past the LDS capacity.
// delta = cdelta*dn/vmax, narrowed in proportion to Tmin while Tmin < r0*dnx/vmax.
#include "kernels.h"
#include "local_ops.h"
#include "fields.h"
#include "band_common.h"

namespace af {


#ifndef AF_THREADS
#define AF_THREADS 512
#endif
constexpr int kThreads = AF_THREADS;
constexpr int kWaves = kThreads / 64;
#ifndef AF_LCAP
#define AF_LCAP 3584
#endif
#ifndef AF_HASH_LOG2
#define AF_HASH_LOG2 13
#endif
#ifndef AF_HASH_ITEMS
#define AF_HASH_ITEMS 6144
#endif
constexpr int kLcap = AF_LCAP, kAcap = 2048, kEcap = 2816;
constexpr int kHash = 1 << AF_HASH_LOG2;    // LDS hash set of claimed cells
constexpr int kHashItems = AF_HASH_ITEMS;  // (load <= 0.75) steps with more claim items use the global stamps
constexpr int kStabLds = 64;    // stiffness rows staged in LDS (more rows: global)
constexpr int kPtabLds = 722;   // phase-table doubles staged in LDS (361 x ncol <= 2 columns)
constexpr int kMatLds = 256;    // material records staged in LDS (DevModel::mtab)

struct BandLds {
  double red[kWaves];
  double Lt[kLcap];  // close set: T of the slot (+inf: free)
  double Vl[kEcap];  // evaluated values
  double stab[kStabLds * 5];
  double ptab[kPtabLds];
  MatRec mat[kMatLds];
  int Ll[kLcap];     // close set: cell of the slot
  int Fs[kLcap];     // free slots
  int Al[kAcap];     // accepted cells
  int El[kEcap];     // claimed cells
  int Ep[kEcap];     // slot of a claimed close cell, -1 for a far cell
  alignas(16) int H[kHash];  // hash set of this step's claimed cells (cell + 1; 0 empty)
  int nA, nE, nF, hi, taken;
  int err;
};

// fouds18_A() fallback (rare)
AF_DEV
double fouds18_global(const GField& F, const DevModel& M, const CellMat& cm, int z, int x, double dnx, double dnz,
                      int nx, int nz, const double* pre) {
  return fouds18(F, M, cm, z, x, dnx, dnz, nx, nz, pre);
}

AF_DEV unsigned hash_slot(int key) { return ((unsigned)key * 2654435761u) >> (32 - AF_HASH_LOG2); }
// probe stride of key (double hashing): odd, so the sequence visits every slot
AF_DEV unsigned hstep(int key) { return (((unsigned)key * 0x85ebca6bu) >> (32 - AF_HASH_LOG2)) | 1u; }

// one band run over the main grid; returns steps.  T/S in global memory, sets and lists in LDS.
// On entry the close set holds slots [0, sh->hi) with sh->nF free slots in sh->Fs.
template <bool LDSMAT>
AF_DEV long long band_run(const BandParams& P, BandLds* sh, BandSrc* B, const RunCfg& R) {
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const int nz = R.nz, nx = R.nx;
  double* T = B->T;
  int* S = B->S;
  int* own = B->own;  // claim stamps (host-initialised to -1)
  const GField F{T, S, nz, nx};
  DevModel M = P.M;
  if (LDSMAT) M.ptab = sh->ptab;
  const HList<int, kLcap> L{sh->Ll, B->L0};
  const HList<double, kLcap> Lt{sh->Lt, B->Lt0};
  const HList<int, kLcap> FS{sh->Fs, B->L1};
  const HList<int, kAcap> AL{sh->Al, B->A};
  const HList<int, kEcap> EL{sh->El, B->C};
  const HList<int, kEcap> EP{sh->Ep, B->Cp};
  const HList<double, kEcap> VL{sh->Vl, B->V};
  long long steps = 0, myupd = 0;
  const bool prof = P.prof && tid == 0;
  long long ph[6] = {0, 0, 0, 0, 0, 0}, ls[3] = {0, 0, 0}, lmax = 0, tk = prof ? wall_clock64() : 0;
  long long sub[4] = {0, 0, 0, 0}, ts = 0;
#define AF_SUB(k)                      \
  if (prof) {                          \
    __builtin_amdgcn_s_waitcnt(0);     \
    long long t_ = wall_clock64();     \
    sub[k] += t_ - ts;                 \
    ts = t_;                           \
  }
#define AF_TICK(k)                 \
  if (prof) {                      \
    long long t_ = wall_clock64(); \
    ph[k] += t_ - tk;              \
    tk = t_;                       \
  }
  while (true) {
    const int hi = sh->hi;
    const int live = hi - sh->nF;
    // ---- phase 1: Tmin over the close set (LDS); clear the hash set ----
    double tmin = INFINITY;
    for (int e = tid; e < hi; e += kThreads) tmin = fmin(tmin, Lt.get(e));
    for (int k = tid * 4; k < kHash; k += kThreads * 4) *(int4*)&sh->H[k] = make_int4(0, 0, 0, 0);
    tmin = wave_min(tmin);
    if (lane == 0) sh->red[wv] = tmin;
    if (tid == 0) {
      sh->nA = 0;
      sh->nE = 0;
      sh->taken = 0;
    }
    __syncthreads();
    AF_TICK(0)
    if (live <= 0) break;
    tmin = sh->red[0];
    for (int w = 1; w < kWaves; w++) tmin = fmin(tmin, sh->red[w]);
    double dl = R.delta;
    if (R.t0 > 0 && tmin < R.t0) dl = R.delta * (tmin / R.t0);
    const double thr = tmin + dl;
    // ---- phase 2: accept (-> known, slot freed) ----
    for (int e0 = wv * 64; e0 < hi; e0 += kThreads) {
      const int e = e0 + lane;
      const double t = e < hi ? Lt.get(e) : INFINITY;
      const bool acc = t <= thr;
      int sa, sf;
      wave_push2(&sh->nA, &sh->nF, acc, P.capL, &sh->err, sa, sf);
      if (sa >= 0) {
        const int c = L.get(e);
        AL.put(sa, c);
        gst(S + pk_flat(c, nx), (int)kKnown);
        Lt.put(e, INFINITY);
        FS.put(sf, e);
      }
    }
    __syncthreads();
    AF_TICK(1)
    const int nA = min(sh->nA, P.capL);
    // ---- phase 3a: claim.  Each distinct neighbour of the accepted cells is owned by one item.
    // Steps with <= kHashItems items dedupe in the LDS hash set; larger steps (long fronts) stamp
    // own[cell] with the step number by a global atomicMax (winner: previous stamp < step).
    const int nItems = 4 * nA;
    const bool use_hash = nItems <= kHashItems;
    const int stamp = (int)steps;
    for (int q0 = wv * 64 * 8; q0 < nItems; q0 += kThreads * 8) {
      int r[8], s[8], o[8];
      if (prof) ts = wall_clock64();
      // first probe of all 8 items issued back to back (one LDS round trip), collisions after
      unsigned hh[8];
      int pv[8];
      if (nA <= kAcap) {  // (uniform) accepted list in LDS: branch-free item generation
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const int q = q0 + u * 64 + lane;
          const int c = nb_cell(AL.lds(q < nItems ? q >> 2 : 0), q & 3, nz, nx);
          r[u] = q < nItems ? c : -1;
          hh[u] = hash_slot(r[u]);
        }
      } else {
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const int q = q0 + u * 64 + lane;
          r[u] = q < nItems ? nb_cell(AL.get(q >> 2), q & 3, nz, nx) : -1;
          hh[u] = hash_slot(r[u]);
        }
      }
      if (use_hash) {
#pragma unroll
        for (int u = 0; u < 8; u++) pv[u] = r[u] >= 0 ? atomicCAS(&sh->H[hh[u]], 0, r[u] + 1) : 0;
        // collisions: double hashing (odd key-dependent stride: no primary clusters), all 8
        // items in ONE loop whose trip count is the longest probe sequence among them
        unsigned pend = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) {
          if (pv[u] != 0) {
            if (pv[u] == r[u] + 1) r[u] = -1;  // already claimed
            else pend |= 1u << u;
          }
        }
        for (int probe = 1; pend; probe++) {
          if (probe >= kHash) {
            sh->err = 5;
#pragma unroll
            for (int u = 0; u < 8; u++)
              if ((pend >> u) & 1u) r[u] = -1;
            break;
          }
#pragma unroll
          for (int u = 0; u < 8; u++) {
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
      AF_SUB(0)
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int f = r[u] >= 0 ? pk_flat(r[u], nx) : 0;
        s[u] = r[u] >= 0 ? gld(S + f) : (int)kKnown;
        o[u] = (!use_hash && r[u] >= 0) ? gatomic_max(own + f, stamp) : -1;
      }
      AF_SUB(1)
      // one list allocation per wave for all 8 items
      // u-major list order: consecutive entries are neighbours of consecutive accepted cells, so
      // the lanes of an evaluating wave read overlapping stencils (fewer distinct cache lines)
      unsigned long long bm[8];
      int cnt = 0;
#pragma unroll
      for (int u = 0; u < 8; u++) {
        bm[u] = __ballot(s[u] != kKnown && o[u] < stamp);
        cnt += __popcll(bm[u]);
      }
      int base = 0;
      if (lane == 0 && cnt) base = atomicAdd(&sh->nE, cnt);
      base = __shfl(base, 0);
      const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if ((bm[u] >> lane) & 1ull) {
          const int pos = base + __popcll(bm[u] & lt);
          if (pos < P.capC) {
            EL.put(pos, r[u]);
            EP.put(pos, s[u] > 0 ? s[u] - 1 : -1);
          } else {
            sh->err = 2;
          }
        }
        base += __popcll(bm[u]);
      }
      AF_SUB(2)
    }
    __syncthreads();
    AF_TICK(2)
    const int nE = min(sh->nE, P.capC);
    // ---- phase 3b: evaluate ----
    const bool lds_e = nE <= kEcap;  // (uniform) the claimed list is in LDS
    for (int e = tid; e < nE; e += kThreads) {
      const int r = lds_e ? EL.lds(e) : EL.get(e);
      const int z = pkz(r), x = pkx(r);
      if (prof) ts = wall_clock64();
      NbFieldT nb;  // stencil loads first, then the material id: one memory round trip
      nb.load(T, nz, nx, z, x);
      const CellMat cm = band_mat<LDSMAT>(M, sh->mat, sh->stab, R.mv, z, x);
      AF_SUB(3)
      const double v = update(nb, M, cm, z, x, R.dnx, nz, nx);
      if (lds_e) VL.put_lds(e, v);
      else VL.put(e, v);
      myupd++;
    }
    AF_TICK(3)
    // fouds18_A() fallback (update() found no usable stencil): a loop of its own, so its live
    // ranges never overlap update()'s
    for (int e = tid; e < nE; e += kThreads) {
      if (VL.get(e) == -1.0) {
        const int r = EL.get(e);
        const int z = pkz(r), x = pkx(r);
        const CellMat cm = band_mat<LDSMAT>(M, sh->mat, sh->stab, R.mv, z, x);
        VL.put(e, fouds18_global(F, M, cm, z, x, R.dnx, R.dnz, nx, nz, mat_slo(M, R.mv, z, x)));
      }
    }
    __syncthreads();
    AF_TICK(4)
    // ---- phase 4: commit; far cells take free slots (top of the stack first), then new ones ----
    const int nF = sh->nF;
    for (int e0 = wv * 64; e0 < nE; e0 += kThreads) {
      const int e = e0 + lane;
      bool fresh = false;
      int r = 0;
      double v = 0.0;
      if (e < nE) {
        r = EL.get(e);
        v = VL.get(e);
        const int p = EP.get(e);
        gst(T + pk_flat(r, nx), v);
        if (p >= 0) Lt.put(p, v);
        else fresh = true;
      }
      const int k = wave_push(&sh->taken, fresh, 1 << 30, &sh->err);
      if (k >= 0) {
        const int slot = k < nF ? FS.get(nF - 1 - k) : hi + (k - nF);
        if (slot >= P.capL) {
          sh->err = 2;
        } else {
          L.put(slot, r);
          Lt.put(slot, v);
          gst(S + pk_flat(r, nx), 1 + slot);
        }
      }
    }
    __syncthreads();
    AF_TICK(5)
    if (tid == 0) {
      const int tk_ = sh->taken;
      sh->nF = max(0, nF - tk_);
      sh->hi = hi + max(0, tk_ - nF);
    }
    if (prof) {
      ls[0] += live;
      ls[1] += nA;
      ls[2] += nE;
      lmax = max(lmax, (long long)hi);
    }
    steps++;
    __syncthreads();
    if (sh->err) break;
  }
  for (int o = 32; o > 0; o >>= 1) myupd += __shfl_xor(myupd, o);
  if (lane == 0 && myupd) atomicAdd((unsigned long long*)&B->nupd, (unsigned long long)myupd);
  if (prof) {
    for (int k = 0; k < 6; k++) B->ph[k] += ph[k];
    for (int k = 0; k < 3; k++) B->lsum[k] += ls[k];
    for (int k = 0; k < 4; k++) B->sub[k] += sub[k];
    B->lmax = max(B->lmax, lmax);
  }
#undef AF_TICK
#undef AF_SUB
  __syncthreads();
  return steps;
}

template <int MODE, bool LDSMAT>
__global__ __launch_bounds__(kThreads) void fmm_band_kernel(BandParams P) {
  __shared__ BandLds sh;
  const int src = blockIdx.x;
  if (src >= P.nsrc) return;
  BandSrc* B = P.src + src;
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  if (tid == 0) {
    sh.hi = 0;
    sh.nF = 0;
    sh.err = 0;
  }
  if (LDSMAT) {
    for (int k = tid; k < 5 * P.M.nstab; k += kThreads) sh.stab[k] = P.M.stab[k];
    for (int k = tid; k < 361 * P.M.ncol; k += kThreads) sh.ptab[k] = P.M.ptab[k];
    for (int k = tid; k < P.M.nmat; k += kThreads) sh.mat[k] = P.M.mtab[k];
  }
  __syncthreads();
  const HList<int, kLcap> L0{sh.Ll, B->L0};
  const HList<double, kLcap> Lt0{sh.Lt, B->Lt0};
  if (MODE == 0) {
    // ---------------- travel(): hand-over of the exact-heap init (fmm_init_kernel) ----------------
    const HandoverOut* H = P.ho + src;
    if (tid == 0) sh.err = H->err ? 3 : 0;
    const int n = H->n;
    for (int k0 = wv * 64; k0 < n; k0 += kThreads) {
      const int k = k0 + lane;
      bool push = false;
      int c = 0;
      double t = 0.0;
      if (k < n) {
        c = H->cell[k];
        t = H->ttn[k];
        gst(B->T + c, t);
        if (H->cls[k] == 1) gst(B->S + c, (int)kKnown);
        else push = true;
      }
      const int s = wave_push(&sh.hi, push, P.capL, &sh.err);
      if (s >= 0) {
        L0.put(s, pk(c / P.nx, c % P.nx));
        Lt0.put(s, t);
        gst(B->S + c, 1 + s);
      }
    }
  } else {
    // ---------------- travel_finer_grid(): stages + exact prefix ran in fmm_exact_kernel ----------------
    if (tid == 0) {
      if (B->err) sh.err = B->err;
      sh.hi = B->nl0;
    }
    for (int k = tid; k < B->nl0; k += kThreads) {
      const int c = gld(B->L0 + k);
      L0.put(k, pk(c / P.nx, c % P.nx));  // (in place: entry k of L0 is read before it is rewritten)
      Lt0.put(k, gld(B->T + c));
    }
  }
  __syncthreads();
  // ---------------- main grid ----------------
  if (!sh.err) {
    RunCfg R;
    R.nz = P.nz;
    R.nx = P.nx;
    R.dnx = P.dnx;
    R.dnz = P.dnz;
    if (MODE == 0)
      R.mv = MatView{1, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0};
    else
      R.mv = MatView{P.sg, (P.sg - 1) / 2, 0, P.sg, (P.sg - 1) / 2, 0, 1, 0, 0, 0, 1};
    R.delta = P.cdelta * P.dnx / P.vmax;
    R.t0 = P.r0 * P.dnx / P.vmax;
    const long long st = band_run<LDSMAT>(P, &sh, B, R);
    if (tid == 0) B->steps[3] = st;
  }
  if (tid == 0) B->err = sh.err;
}

// final scaling of travel_finer_grid (:2832 ttn / subgrid_size)
__global__ void scale_kernel(double* T, long n, double inv) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) T[i] = T[i] / inv;
}

}  // namespace af

extern "C" hipError_t af_launch_band(const af::BandParams* P, hipStream_t stream) {
  const bool lds = P->M.mid && P->M.nmat <= af::kMatLds && P->M.nstab <= af::kStabLds &&
                   361 * P->M.ncol <= af::kPtabLds;
  // (mode 1 hands over fmm_exact_kernel's close list in L0; the band run keeps it there)
  const dim3 g(P->nsrc), b(af::kThreads);
  if (P->mode == 0) {
    if (lds) hipLaunchKernelGGL((af::fmm_band_kernel<0, true>), g, b, 0, stream, *P);
    else hipLaunchKernelGGL((af::fmm_band_kernel<0, false>), g, b, 0, stream, *P);
  } else {
    if (lds) hipLaunchKernelGGL((af::fmm_band_kernel<1, true>), g, b, 0, stream, *P);
    else hipLaunchKernelGGL((af::fmm_band_kernel<1, false>), g, b, 0, stream, *P);
  }
  return hipGetLastError();
}

extern "C" hipError_t af_launch_scale(double* T, long n, double sg, hipStream_t stream) {
  hipLaunchKernelGGL(af::scale_kernel, dim3(2048), dim3(256), 0, stream, T, n, sg);
  return hipGetLastError();
}
