// fmm_band.hip — band-synchronous ("Delta-stepping") FMM on gfx950.
//
// Replaces the reference's heap-ordered main loop (travel :2055-2102, travel_finer_grid
// :2775-2817).  One persistent 1024-thread workgroup per source; all synchronisation is
// workgroup-local (s_barrier), so sources never wait on each other.  Per step:
//   1  Tmin over the close list (wave DPP min + LDS)                       [T gather]
//   2  accept every close cell with T <= Tmin + delta(Tmin) -> known, compact the rest
//   3  for each (accepted cell, direction): claim the neighbour with one atomicCAS on its
//      status (far->far_cand / close->close_cand; claims never change update() validity),
//      evaluate the reference's update() (fallback fouds18_A()) against the post-acceptance
//      state, Jacobi-style, into the candidate list
//   4  commit: T <- new value, status -> close, new close cells appended to the list
// Lists are appended with one LDS atomic per wave (ballot + mbcnt).  delta = cdelta*dn/vmax,
// narrowed in proportion to Tmin while Tmin < r0*dnx/vmax (near-source schedule).
// The same routine runs the refined stage grids of travel_finer_grid (mode 1).
#include "kernels.h"
#include "local_ops.h"
#include "fields.h"

namespace af {



constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
// LDS-resident heads of the per-step lists; entries past the cap spill to the global arrays of
// the same index (BandSrc L0/L1, A, C, V), so LDS bounds only speed, never capacity.
constexpr int kLcap = 6144, kAcap = 4096, kEcap = 6144;

struct BandLds {
  double red[kWaves];
  double Vl[kEcap];
  int cnt[2][3];  // [parity][A, L2, E]
  int finished;
  int err;
  int Ll[2][kLcap];
  int Al[kAcap];
  int El[kEcap];
};

template <int CAP>
struct HList {
  int* l;  // LDS head
  int* g;  // global array (same indexing)
  AF_DEV int get(int i) const { return i < CAP ? l[i] : g[i]; }
  AF_DEV void put(int i, int v) const {
    if (i < CAP) l[i] = v;
    else g[i] = v;
  }
};
typedef HList<kLcap> LList;

AF_DEV int lane_id() { return threadIdx.x & 63; }

// append with one LDS atomic per wave; returns the slot or -1 (pred false / overflow)
AF_DEV int wave_push(int* counter, bool pred, int cap, int* err) {
  unsigned long long m = __ballot(pred);
  if (m == 0) return -1;
  int lane = lane_id();
  int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader);
  int off = __popcll(m & ((1ull << lane) - 1ull));
  if (!pred) return -1;
  int slot = base + off;
  if (slot >= cap) {
    *err = 2;
    return -1;
  }
  return slot;
}

AF_DEV double wave_min(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  return v;
}

struct RunCfg {
  int nz, nx;
  double dnx, dnz;  // update() spacing and fouds18 dnz
  MatView mv;
  int stage;        // window-edge finish test enabled
  int isx, isz, max_dist;
  double delta, t0;
};

AF_DEV LList band_list(BandLds* sh, BandSrc* B, int k) { return LList{sh->Ll[k], k ? B->L1 : B->L0}; }

// one band run; returns steps.  T/S in global memory, list heads and counts in LDS.
// lc: index (0/1) of the list holding the nL close cells on entry and on return.
AF_DEV long long band_run(const BandParams& P, BandLds* sh, BandSrc* B, double* T, int* S, int& lc, int& nL,
                          const RunCfg& R, long long* nupd) {
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const int nz = R.nz, nx = R.nx;
  const long ncell = (long)nz * nx;
  const GField F{T, S, nz, nx};
  const HList<kAcap> AL{sh->Al, B->A};
  const HList<kEcap> EL{sh->El, B->C};
  long long steps = 0;
  long long myupd = 0;
  if (tid == 0) {
    sh->finished = 0;
    for (int p = 0; p < 2; p++)
      for (int q = 0; q < 3; q++) sh->cnt[p][q] = 0;
  }
  __syncthreads();
  while (true) {
    const int par = (int)(steps & 1);
    const LList L = band_list(sh, B, lc), L2 = band_list(sh, B, lc ^ 1);
    // ---- phase 1: Tmin over the close list (4 gathers in flight per lane) ----
    double tmin = INFINITY;
    for (int e0 = tid; e0 < nL; e0 += 4 * kThreads) {
      int c[4];
      double t[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        int e = e0 + u * kThreads;
        c[u] = e < nL ? L.get(e) : -1;
      }
#pragma unroll
      for (int u = 0; u < 4; u++) t[u] = T[c[u] < 0 ? 0 : c[u]];
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (c[u] >= 0) tmin = fmin(tmin, t[u]);
    }
    tmin = wave_min(tmin);
    if (lane == 0) sh->red[wv] = tmin;
    __syncthreads();
    tmin = sh->red[0];
    for (int w = 1; w < kWaves; w++) tmin = fmin(tmin, sh->red[w]);
    if (nL == 0) break;
    double dl = R.delta;
    if (R.t0 > 0 && tmin < R.t0) dl = R.delta * (tmin / R.t0);
    const double thr = tmin + dl;
    int* cA = &sh->cnt[par][0];
    int* cL2 = &sh->cnt[par][1];
    int* cE = &sh->cnt[par][2];
    // ---- phase 2: accept / compact ----
    for (int e0 = wv * 64; e0 < nL; e0 += 2 * kThreads) {
      int c[2];
      double t[2];
#pragma unroll
      for (int u = 0; u < 2; u++) {
        int e = e0 + u * kThreads + lane;
        c[u] = e < nL ? L.get(e) : -1;
      }
#pragma unroll
      for (int u = 0; u < 2; u++) t[u] = T[c[u] < 0 ? 0 : c[u]];
#pragma unroll
      for (int u = 0; u < 2; u++) {
        bool valid = c[u] >= 0;
        bool acc = valid && t[u] <= thr;
        if (acc) S[c[u]] = kKnown;
        int sa = wave_push(cA, acc, P.capL, &sh->err);
        if (sa >= 0) AL.put(sa, c[u]);
        int sl = wave_push(cL2, valid && !acc, P.capL, &sh->err);
        if (sl >= 0) L2.put(sl, c[u]);
      }
    }
    __syncthreads();
    const int nA = min(*cA, P.capL);
    if (tid == 0) {  // reset the other parity's counters (read by everyone before this step's barrier)
      sh->cnt[par ^ 1][0] = 0;
      sh->cnt[par ^ 1][1] = 0;
      sh->cnt[par ^ 1][2] = 0;
    }
    // ---- phase 3a: claim the neighbours of the accepted cells (far->far_cand, close->close_cand) ----
    const int nItems = 4 * nA;
    for (int q0 = wv * 64; q0 < nItems; q0 += kThreads) {
      int q = q0 + lane;
      bool won = false;
      int r = 0;
      if (q < nItems) {
        int a = AL.get(q >> 2), dir = q & 3;
        int iz = a / nx, ix = a - iz * nx;
        int z = iz + (dir == 2 ? -1 : dir == 3 ? 1 : 0);
        int x = ix + (dir == 0 ? -1 : dir == 1 ? 1 : 0);
        if (z < 0 || z >= nz || x < 0 || x >= nx) {
          if (R.stage) {
            // window-edge finish test (:1651-1652, :1673-1674)
            if (dir < 2 ? (abs(R.isx - x) == R.max_dist + 1) : (abs(R.isz - z) == R.max_dist + 1))
              sh->finished = 1;
          }
        } else {
          r = z * nx + x;
          int s = S[r];
          bool fresh = false;
          if (s == kFar) fresh = won = atomicCAS(&S[r], kFar, kFarCand) == kFar;
          else if (s == kClose) won = atomicCAS(&S[r], kClose, kCloseCand) == kClose;
          if (fresh) r = -(r + 1);  // far -> close: remembered here, never re-read from S (L1 may be stale)
        }
      }
      int se = wave_push(cE, won, P.capC, &sh->err);
      if (se >= 0) EL.put(se, r);
    }
    __syncthreads();
    const int nE = min(*cE, P.capC);
    // ---- phase 3b: evaluate (Jacobi against the post-acceptance state), all lanes busy ----
    for (int e = tid; e < nE; e += kThreads) {
      int r = EL.get(e);
      if (r < 0) r = -r - 1;
      int z = r / nx, x = r - z * nx;
      CellMat cm = cell_mat(P.M, R.mv, z, x);
      NbField nb;
      nb.load(T, S, nz, nx, z, x);
      double v = update(nb, P.M, cm, z, x, R.dnx, nz, nx);
      if (e < kEcap) sh->Vl[e] = v;
      else B->V[e] = v;
      myupd++;
    }
    // fouds18_A() fallback (update() found no usable stencil): a loop of its own over the same
    // entries, so its live ranges never overlap update()'s (no register spills)
    for (int e = tid; e < nE; e += kThreads) {
      double v = e < kEcap ? sh->Vl[e] : B->V[e];
      if (v == -1.0) {
        int r = EL.get(e);
        if (r < 0) r = -r - 1;
        int z = r / nx, x = r - z * nx;
        CellMat cm = cell_mat(P.M, R.mv, z, x);
        v = fouds18(F, P.M, cm, z, x, R.dnx, R.dnz, nx, nz);
        if (e < kEcap) sh->Vl[e] = v;
        else B->V[e] = v;
      }
    }
    __syncthreads();
    // ---- phase 4: commit (same lane <-> entry map as 3b) ----
    for (int e0 = wv * 64; e0 < nE; e0 += kThreads) {
      int e = e0 + lane;
      bool fresh = false;
      int r = 0;
      if (e < nE) {
        r = EL.get(e);
        fresh = r < 0;
        if (fresh) r = -r - 1;
        T[r] = e < kEcap ? sh->Vl[e] : B->V[e];
        S[r] = kClose;
      }
      int sl = wave_push(cL2, fresh, P.capL, &sh->err);
      if (sl >= 0) L2.put(sl, r);
    }
    __syncthreads();
    nL = min(*cL2, P.capL);
    lc ^= 1;
    steps++;
    if (sh->finished || sh->err) break;
  }
  if (nupd) {
    for (int o = 32; o > 0; o >>= 1) myupd += __shfl_xor(myupd, o);
    if (lane == 0 && myupd) atomicAdd((unsigned long long*)nupd, (unsigned long long)myupd);
  }
  __syncthreads();
  (void)ncell;
  return steps;
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void fmm_band_kernel(BandParams P) {
  __shared__ BandLds sh;
  const int src = blockIdx.x;
  if (src >= P.nsrc) return;
  BandSrc* B = P.src + src;
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  if (tid == 0) {
    for (int p = 0; p < 2; p++)
      for (int q = 0; q < 3; q++) sh.cnt[p][q] = 0;
    sh.err = 0;
    sh.finished = 0;
  }
  __syncthreads();
  int lc = 0;
  int nL = 0;
  const double t0 = P.r0 * P.dnx / P.vmax;

  if (MODE == 0) {
    // ---------------- travel(): hand-over of the exact-heap stage 3 (fmm_init_kernel) ----------------
    const HandoverOut* H = P.ho + src;
    if (tid == 0) sh.err = H->err ? 3 : 0;
    const int n = H->n;
    for (int k0 = wv * 64; k0 < n; k0 += kThreads) {
      int k = k0 + lane;
      bool push = false;
      int c = 0;
      if (k < n) {
        c = H->cell[k];
        B->T[c] = H->ttn[k];
        B->S[c] = H->cls[k] == 1 ? kKnown : kClose;
        push = H->cls[k] != 1;
      }
      int s = wave_push(&sh.cnt[1][1], push, P.capL, &sh.err);
      if (s >= 0) band_list(&sh, B, lc).put(s, c);
    }
    __syncthreads();
    nL = sh.cnt[1][1];
    __syncthreads();
    if (tid == 0) sh.cnt[1][1] = 0;
    __syncthreads();
  } else {
    // ---------------- travel_finer_grid(): stages + exact prefix ran in fmm_exact_kernel ----------------
    if (tid == 0 && B->err) sh.err = B->err;
    nL = B->nl0;
    for (int k = tid; k < min(nL, kLcap); k += kThreads) sh.Ll[0][k] = B->L0[k];
    __syncthreads();
  }
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
    R.stage = 0;
    R.isx = R.isz = R.max_dist = 0;
    R.delta = P.cdelta * P.dnx / P.vmax;
    R.t0 = t0;
    long long st = band_run(P, &sh, B, B->T, B->S, lc, nL, R, &B->nupd);
    if (tid == 0) B->steps[3] = st;
  }
  if (tid == 0) B->err = sh.err;
}

// final scaling of travel_finer_grid (:2832 ttn / subgrid_size) fused with nothing else: one pass
__global__ void scale_kernel(double* T, long n, double inv) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) T[i] = T[i] / inv;
}

}  // namespace af

extern "C" hipError_t af_launch_band(const af::BandParams* P, hipStream_t stream) {
  if (P->mode == 0)
    hipLaunchKernelGGL(af::fmm_band_kernel<0>, dim3(P->nsrc), dim3(af::kThreads), 0, stream, *P);
  else
    hipLaunchKernelGGL(af::fmm_band_kernel<1>, dim3(P->nsrc), dim3(af::kThreads), 0, stream, *P);
  return hipGetLastError();
}

extern "C" hipError_t af_launch_scale(double* T, long n, double sg, hipStream_t stream) {
  hipLaunchKernelGGL(af::scale_kernel, dim3(2048), dim3(256), 0, stream, T, n, sg);
  return hipGetLastError();
}
