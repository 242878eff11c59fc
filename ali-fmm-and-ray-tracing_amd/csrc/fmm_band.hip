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

namespace af {



constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;

struct GField {
  const double* T;
  const int* S;
  int nz, nx;
  AF_DEV int st(long z, long x) const { return z >= nz ? -1 : S[z * nx + x]; }
  AF_DEV double tt(long z, long x) const { return z >= nz ? 0.0 : T[z * nx + x]; }
};

struct BandLds {
  double red[kWaves];
  int cnt[2][3];  // [parity][A, L2, C]
  int finished;
  int err;
};

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

// one band run; returns steps.  T/S/lists in global memory, counts in LDS.
AF_DEV long long band_run(const BandParams& P, BandLds* sh, double* T, int* S, int*& L, int*& L2, int& nL, int* A,
                          int* C, double* V, const RunCfg& R, long long* nupd) {
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const int nz = R.nz, nx = R.nx;
  const GField F{T, S, nz, nx};
  long long steps = 0;
  if (tid == 0) {
    sh->finished = 0;
    for (int p = 0; p < 2; p++)
      for (int q = 0; q < 3; q++) sh->cnt[p][q] = 0;
  }
  __syncthreads();
  while (true) {
    const int par = (int)(steps & 1);
    // ---- phase 1: Tmin over the close list ----
    double tmin = INFINITY;
    for (int e = tid; e < nL; e += kThreads) tmin = fmin(tmin, T[L[e]]);
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
    int* cC = &sh->cnt[par][2];
    // ---- phase 2: accept / compact ----
    for (int e0 = wv * 64; e0 < nL; e0 += kThreads) {
      int e = e0 + lane;
      bool valid = e < nL;
      int c = valid ? L[e] : 0;
      double t = valid ? T[c] : 0.0;
      bool acc = valid && t <= thr;
      if (acc) S[c] = kKnown;
      int sa = wave_push(cA, acc, P.capL, &sh->err);
      if (sa >= 0) A[sa] = c;
      int sl = wave_push(cL2, valid && !acc, P.capL, &sh->err);
      if (sl >= 0) L2[sl] = c;
    }
    __syncthreads();
    const int nA = *cA;
    if (tid == 0) {  // reset the other parity's counters (read by everyone before this step's barrier)
      sh->cnt[par ^ 1][0] = 0;
      sh->cnt[par ^ 1][1] = 0;
      sh->cnt[par ^ 1][2] = 0;
    }
    // ---- phase 3: claim + evaluate (Jacobi against the post-acceptance state) ----
    const int nItems = 4 * nA;
    long long myupd = 0;
    for (int q0 = wv * 64; q0 < nItems; q0 += kThreads) {
      int q = q0 + lane;
      bool won = false;
      int r = 0;
      double v = 0.0;
      if (q < nItems) {
        int a = A[q >> 2], dir = q & 3;
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
          if (won) {
            CellMat cm = cell_mat(P.M, R.mv, z, x);
            v = update(F, P.M, cm, z, x, R.dnx, nz, nx);
            if (v == -1.0) v = fouds18(F, P.M, cm, z, x, R.dnx, R.dnz, nx, nz);
            myupd++;
          }
        }
      }
      int sc = wave_push(cC, won, P.capC, &sh->err);
      if (sc >= 0) {
        C[sc] = r;
        V[sc] = v;
      }
    }
    if (nupd) {
      for (int o = 32; o > 0; o >>= 1) myupd += __shfl_xor(myupd, o);
      if (lane == 0 && myupd) atomicAdd((unsigned long long*)nupd, (unsigned long long)myupd);
    }
    __syncthreads();
    const int nC = *cC;
    // ---- phase 4: commit ----
    for (int k0 = wv * 64; k0 < nC; k0 += kThreads) {
      int k = k0 + lane;
      bool valid = k < nC;
      bool fresh = false;
      int r = 0;
      if (valid) {
        r = C[k];
        fresh = r < 0;
        if (fresh) r = -r - 1;
        T[r] = V[k];
        S[r] = kClose;
      }
      int sl = wave_push(cL2, fresh, P.capL, &sh->err);
      if (sl >= 0) L2[sl] = r;
    }
    __syncthreads();
    nL = *cL2;
    int* t = L;
    L = L2;
    L2 = t;
    steps++;
    if (sh->finished || sh->err) break;
  }
  __syncthreads();
  return steps;
}

// ------------------------------------------------------------------------------------------------
// hand-over of a (band) stage grid into the next grid (:2391-2425, :2725-2759): every 3rd node
AF_DEV void band_handover(BandLds* sh, const double* sT, const int* sS, int snz, int snx, int isz_s, int isx_s,
                          double* dT, int* dS, int dnx_, int isz_d, int isx_d, int* L, int& nL, int cap,
                          int* counter) {
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const int dz = (snz - 1) / 3 + 1, dx = (snx - 1) / 3 + 1, n = dz * dx;
  if (tid == 0) *counter = 0;
  __syncthreads();
  for (int k0 = wv * 64; k0 < n; k0 += kThreads) {
    int k = k0 + lane;
    bool push = false;
    int di = 0;
    if (k < n) {
      int i = 3 * (k / dx), j = 3 * (k % dx);
      int pz = isz_d + (i - isz_s) / 3, px = isx_d + (j - isx_s) / 3;
      di = pz * dnx_ + px;
      int st = sS[i * snx + j];
      dT[di] = sT[i * snx + j];
      if (st == kKnown) {
        bool outer = false;
        if (i - 3 >= 0) { if (sS[(i - 3) * snx + j] == kFar) outer = true; } else outer = true;
        if (i + 3 <= snz - 1) { if (sS[(i + 3) * snx + j] == kFar) outer = true; } else outer = true;
        if (j - 3 >= 0) { if (sS[i * snx + j - 3] == kFar) outer = true; } else outer = true;
        if (j + 3 <= snx - 1) { if (sS[i * snx + j + 3] == kFar) outer = true; } else outer = true;
        dS[di] = outer ? kClose : kKnown;
        push = outer;
      } else if (st > 0) {
        dS[di] = kClose;
        push = true;
      }
    }
    int s = wave_push(counter, push, cap, &sh->err);
    if (s >= 0) L[s] = di;
  }
  __syncthreads();
  nL = *counter;
  __syncthreads();
}

AF_DEV void fill_grid(double* T, int* S, int n) {
  for (int k = threadIdx.x; k < n; k += kThreads) {
    T[k] = 0.0;
    S[k] = kFar;
  }
}

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
  int* L = B->L0;
  int* L2 = B->L1;
  int nL = 0;
  const double t0 = P.r0 * P.dnx / P.vmax;

  if (P.mode == 0) {
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
      if (s >= 0) L[s] = c;
    }
    __syncthreads();
    nL = sh.cnt[1][1];
    __syncthreads();
    if (tid == 0) sh.cnt[1][1] = 0;
    __syncthreads();
  } else {
    // ---------------- travel_finer_grid(): band stages x9, x3 (:2187-2504) ----------------
    const int sg = P.sg;
    const long isx = (long)sg * (long)rint((P.scx[src] - P.gox) / P.dnx);
    const long isz = (long)sg * (long)rint((P.scz[src] - P.goz) / P.dnz);
    const int nnz = P.nz, nnx = P.nx;
    const int size1 = 2 * sg + (sg - 1) / 2, s1 = 9;
    const int size2 = size1 + 3 * sg, s2 = 3;
    const int sgside = (sg - 1) / 2;
    int pisz = 0, pisx = 0, pnz = 0, pnx = 0;
    for (int stg = 0; stg < 2; stg++) {
      const int scale = stg == 0 ? s1 : s2, size = stg == 0 ? size1 : size2;
      const int left = max(0L, isx - size), right = min((long)nnx - 1, isx + size);
      const int bottom = max(0L, isz - size), top = min((long)nnz - 1, isz + size);
      const int nz = scale * (top - bottom) + 1, nx = scale * (right - left) + 1;
      if (nz * nx > P.capS) {
        if (tid == 0) sh.err = 4;
        break;
      }
      const int isx_s = scale * (int)(isx - left), isz_s = scale * (int)(isz - bottom);
      double* Ts = B->Ts[stg & 1];
      int* Ss = B->Ss[stg & 1];
      fill_grid(Ts, Ss, nz * nx);
      __syncthreads();
      RunCfg R;
      R.nz = nz;
      R.nx = nx;
      R.dnx = P.dnx / scale;
      R.dnz = R.dnx;
      R.mv = MatView{scale, (scale - 1) / 2, bottom, scale, (scale - 1) / 2, left, sg, sgside, 0, 0, 1};
      R.stage = 1;
      R.isx = isx_s;
      R.isz = isz_s;
      R.max_dist = scale * size;
      R.delta = P.cdelta * R.dnx / P.vmax;
      R.t0 = t0;
      if (stg == 0) {
        // straight rays (:2223-2267; note veln + angle, SURVEY B-D5) on the fine cell of the source
        const int side1 = (s1 - 1) / 2 + s1 * ((sg - 1) / 2);
        MatView fine{sg, sgside, 0, sg, sgside, 0, 1, 0, 0, 0, 1};
        CellMat cs = cell_mat(P.M, fine, (int)isz, (int)isx);
        const int w = 2 * side1 + 1;
        for (int k = tid; k < w * w; k += kThreads) {
          int i = k / w - side1, j = k % w - side1;
          if (0 <= isz_s + i && isz_s + i <= nz - 1 && 0 <= isx_s + j && isx_s + j <= nx - 1) {
            double angle = (j == 0) ? 90.0 : atan((double)i / (double)j) * kRad2Deg;
            double eff = pymod(cs.veln + angle, 180);
            double velocity = (cs.velpn != 0 || cs.stif == nullptr)
                                  ? table_vel(P.M.gtab, P.M.ncol, eff, cs.velpn, cs.vm)
                                  : christoffel_group(cs.stif, eff, cs.vm);
            double length = R.dnx * sqrt((double)(i * i + j * j));
            Ts[(isz_s + i) * nx + isx_s + j] = length / velocity;
            Ss[(isz_s + i) * nx + isx_s + j] = kKnown;
          }
        }
        __syncthreads();
        // window border of the straight-ray square -> close (:2277-2288)
        const int ne = 4 * w;
        for (int k0 = wv * 64; k0 < ne; k0 += kThreads) {
          int k = k0 + lane;
          bool push = false;
          int c = 0;
          if (k < ne) {
            int side = k / w, t = k % w - side1;
            int z = 0, x = 0;
            bool ok = false;
            if (side == 0) { z = isz_s - side1; x = isx_s + t; ok = z >= 0; }
            else if (side == 1) { z = isz_s + side1; x = isx_s + t; ok = z <= nz - 1; }
            else if (side == 2) { z = isz_s + t; x = isx_s - side1; ok = x >= 0; }
            else { z = isz_s + t; x = isx_s + side1; ok = x <= nx - 1; }
            ok = ok && z >= 0 && z <= nz - 1 && x >= 0 && x <= nx - 1;
            if (ok) {
              c = z * nx + x;
              push = atomicCAS(&Ss[c], kKnown, kClose) == kKnown;
            }
          }
          int s = wave_push(&sh.cnt[1][1], push, P.capL, &sh.err);
          if (s >= 0) L[s] = c;
        }
        __syncthreads();
        nL = sh.cnt[1][1];
        __syncthreads();
        if (tid == 0) sh.cnt[1][1] = 0;
        __syncthreads();
      } else {
        band_handover(&sh, B->Ts[0], B->Ss[0], pnz, pnx, pisz, pisx, Ts, Ss, nx, isz_s, isx_s, L, nL, P.capL,
                      &sh.cnt[1][1]);
        if (tid == 0) sh.cnt[1][1] = 0;
        __syncthreads();
      }
      long long st = band_run(P, &sh, Ts, Ss, L, L2, nL, B->A, B->C, B->V, R, nullptr);
      if (tid == 0) B->steps[stg] = st;
      pisz = isz_s;
      pisx = isx_s;
      pnz = nz;
      pnx = nx;
      if (sh.err) break;
    }
    if (!sh.err) {
      band_handover(&sh, B->Ts[1], B->Ss[1], pnz, pnx, pisz, pisx, B->T, B->S, P.nx, (int)isz, (int)isx, L, nL,
                    P.capL, &sh.cnt[1][1]);
      if (tid == 0) sh.cnt[1][1] = 0;
      __syncthreads();
    }
  }
  // ---------------- main grid ----------------
  if (!sh.err) {
    RunCfg R;
    R.nz = P.nz;
    R.nx = P.nx;
    R.dnx = P.dnx;
    R.dnz = P.dnz;
    if (P.mode == 0)
      R.mv = MatView{1, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0};
    else
      R.mv = MatView{P.sg, (P.sg - 1) / 2, 0, P.sg, (P.sg - 1) / 2, 0, 1, 0, 0, 0, 1};
    R.stage = 0;
    R.isx = R.isz = R.max_dist = 0;
    R.delta = P.cdelta * P.dnx / P.vmax;
    R.t0 = t0;
    long long st = band_run(P, &sh, B->T, B->S, L, L2, nL, B->A, B->C, B->V, R, &B->nupd);
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
  hipLaunchKernelGGL(af::fmm_band_kernel, dim3(P->nsrc), dim3(af::kThreads), 0, stream, *P);
  return hipGetLastError();
}

extern "C" hipError_t af_launch_scale(double* T, long n, double sg, hipStream_t stream) {
  hipLaunchKernelGGL(af::scale_kernel, dim3(2048), dim3(256), 0, stream, T, n, sg);
  return hipGetLastError();
}
