// fmm_exact.hip — the source stages of travel_finer_grid() (Anis_TTF_rays.py:2187-2504) and the
// first part of its fine-grid main loop (:2775-2817), solved exactly as the reference does, on gfx950.
//
// Near the source the reference's heap (round-half-even parent, SURVEY B-D3) pops nodes out of
// time order, and the hand-over nodes and grid edges make the field depend on that order; a
// time-ordered (band) solver differs there by up to a few per cent.  This kernel replays the
// reference's heap walk: x9 stage grid, x3 stage grid, then the fine main grid until the heap
// root reaches P.tstop.  The stage grids (up to 397 x 397 for subgrid 9) and the main grid live
// in HBM; the heap itself (cells + keys, i.e. copies of ttn at insertion/update) lives in LDS, so
// every sift is LDS-only and each pop costs the <= 4 neighbour evaluations (one round trip of
// 24 prefetched loads each, NbField).  One workgroup (one wave) per source; the walk is serial
// (lane 0), the other lanes clear grids and fill the straight-ray footprint.
//
// Output for the band kernel: main-grid statuses known 0 / close 1 + list slot / far -1 and the
// close cells in Lin (count in BandSrc::nl0).
#define CR_LDS_TABLES  // cr_math.h tables in LDS (crm::lds_init at kernel start)
#include "kernels.h"
#include "local_ops.h"
#include "fields.h"

namespace af {

constexpr int kXHeap = 8192;

constexpr int kXSpec = 64;   // speculative relaxations (one per lane)
constexpr int kXLog = 256;   // ring of the last relaxed nodes (the modifications update() can see)

struct XSpec {
  int cell;  // -1: empty
  int ver;   // modifications logged when it was evaluated
  double val;
  UpdSel sel;
};

struct XLds {
  double key[kXHeap];
  int cell[kXHeap];
  XSpec spec[kXSpec];
  int logc[kXLog];
  int dup[8];  // XHeap's nodes with two heap entries (here, not in XHeap: see InitLds::dup)
};

// addtree / updtree / downtree (:94-237) over a global nsts array, heap slots in LDS.  Keys are
// copies of ttn; a node with two heap entries (the stage-1 window corners, added by two of the
// edge loops :2277-2288) has every entry's key refreshed when its ttn changes (dup / sync), as
// the reference's comparisons read the live ttn.
constexpr int kXDup = 8;
struct XHeap {
  XLds* H;
  int* S;
  const double* T;
  int ntr;
  int err;
  int ndup = 0;
  AF_DEV void setS(int c, int v) { S[c] = v; }
  AF_DEV static int parent(int t) { return (int)rint((double)t / 2.0); }  // half-even (:123)
  AF_DEV void swap(int a, int b) {
    int c = H->cell[a];
    H->cell[a] = H->cell[b];
    H->cell[b] = c;
    double k = H->key[a];
    H->key[a] = H->key[b];
    H->key[b] = k;
  }
  AF_DEV void sift_up(int c, int tpc) {
    int tpp = parent(tpc);
    const double tv = H->key[tpc];
    while (tpp > 0) {
      if (tv < H->key[tpp]) {
        setS(c, tpp);
        setS(H->cell[tpp], tpc);
        swap(tpc, tpp);
        tpc = tpp;
        tpp = parent(tpc);
      } else {
        tpp = 0;
      }
    }
  }
  // key = the node's ttn; the relaxation passes the value it has just stored (no reload of T[c]);
  // fresh: the node is known to be far (a relaxation of a far neighbour)
  AF_DEV void add(int c, double key, bool fresh = false) {
    ntr += 1;
    if (ntr >= kXHeap) {
      err = 3;
      ntr = kXHeap - 1;
      return;
    }
    if (!fresh && S[c] > 0) {  // already in the heap: a second entry
      if (ndup == kXDup) {
        err = 3;
        return;
      }
      H->dup[ndup++] = c;
    }
    setS(c, ntr);
    H->cell[ntr] = c;
    H->key[ntr] = key;
    sift_up(c, ntr);
  }
  AF_DEV void add(int c) { add(c, T[c]); }
  // tpc: the node's heap index (its status, read by the caller before the relaxation)
  AF_DEV void upd(int c, int tpc, double key) {
    H->key[tpc] = key;
    sift_up(c, tpc);
  }
  // node c's ttn is now key: every heap entry of a node with two entries takes it
  AF_DEV void sync(int c, double key) {
    bool d = false;
    for (int k = 0; k < ndup; k++) d |= H->dup[k] == c;
    if (!d) return;
    for (int k = 1; k <= ntr; k++)
      if (H->cell[k] == c) H->key[k] = key;
  }
  AF_DEV void down() {
    if (ntr == 1) {
      ntr -= 1;
      return;
    }
    setS(H->cell[ntr], 1);
    H->cell[1] = H->cell[ntr];
    H->key[1] = H->key[ntr];
    ntr -= 1;
    int tpp = 1, tpc = 2;
    while (tpc < ntr) {
      if (H->key[tpc] > H->key[tpc + 1]) tpc = tpc + 1;
      if (H->key[tpc] < H->key[tpp]) {
        setS(H->cell[tpp], tpc);
        setS(H->cell[tpc], tpp);
        swap(tpc, tpp);
        tpp = tpc;
        tpc = 2 * tpp;
      } else {
        tpc = ntr + 1;
      }
    }
    if (tpc == ntr) {
      if (H->key[tpc] < H->key[tpp]) {
        setS(H->cell[tpp], tpc);
        setS(H->cell[tpc], tpp);
        swap(tpc, tpp);
      }
    }
  }
};

struct XGrid {
  double* T;
  int* S;
  int nz, nx;
  MatView mv;
  double dnx, dnz;  // update() spacing, fouds18 dnz
};

// bounding box of the nodes written into a grid ({z0, z1, x0, x1}; empty: z0 > z1)
struct XBox {
  int b[4] = {1 << 30, -1, 1 << 30, -1};
  AF_DEV void add(int z, int x) {
    b[0] = min(b[0], z);
    b[1] = max(b[1], z);
    b[2] = min(b[2], x);
    b[3] = max(b[3], x);
  }
};

// The walk with relaxations evaluated ahead of their turn (the HBM-grid counterpart of
// fmm_init.hip's relax_role): when a neighbour's relaxation has no usable entry, the wavefront
// runs one pass in which lane 0 evaluates it and every other lane a neighbour of one of the heap's
// first 16 entries (the next pops), all against the current state (one round of stencil loads).
// An entry stays usable while no node of its 12-point stencil has been relaxed since it was
// evaluated: every relaxation is logged (XLds::logc), and the lanes check the log since the entry's
// version in parallel.  update() reads nothing but those 12 nodes' values and validity, so a
// usable entry's value is the relaxation's value bit for bit; statuses changing from close to
// known (pops) are not logged — update() does not distinguish them — and fouds18_A() (no usable
// stencil: known-ness matters) always runs in turn.  Returns the pops (lane 0's count).
AF_DEV long long xloop_spec(XHeap& h, const DevModel& M, const XGrid& g, bool stage, int isx_s, int isz_s,
                            int max_dist, double tstop, XBox* box, int lane, long long* prof = nullptr) {
  long long pops = 0;
  bool finished = false;
  const int nz = g.nz, nx = g.nx;
  XLds* X = h.H;
  int mver = 0;  // relaxations logged (wave-uniform)
  long long npass = 0;
  X->spec[lane].cell = -1;
  while (true) {
    int go = 0, c = 0;
    if (lane == 0) {
      go = h.ntr > 0 && !finished && !h.err && !(tstop > 0 && h.H->key[1] >= tstop);
      c = h.H->cell[1];
    }
    go = __shfl(go, 0);
    if (!go) break;
    c = __shfl(c, 0);
    const int iz = c / nx, ix = c - iz * nx;
    // lane k < 4: neighbour k (x-1, x+1, z-1, z+1); its status is read before downtree: downtree and
    // the add / upd of earlier neighbours only move heap indices (positive stays positive) and touch
    // no other neighbour's far / known state, so the reference's per-neighbour classification
    // (far -1 -> add, close > 0 -> upd, known 0 -> skip) can be read up front
    const int kz = lane == 2 ? iz - 1 : lane == 3 ? iz + 1 : iz;
    const int kx = lane == 0 ? ix - 1 : lane == 1 ? ix + 1 : ix;
    const bool inb = lane < 4 && (lane < 2 ? (0 <= kx && kx <= nx - 1) : (0 <= kz && kz <= nz - 1));
    const int st = inb ? g.S[kz * nx + kx] : 0;
    const bool edge = lane < 4 && !inb && stage && (lane < 2 ? abs(isx_s - kx) : abs(isz_s - kz)) == max_dist + 1;
    const unsigned long long jm = __ballot(inb && st != 0);
    if (__ballot(edge) != 0ull) finished = true;
    int stk[4];
#pragma unroll
    for (int k = 0; k < 4; k++) stk[k] = __shfl(st, k);
    if (lane == 0) {
      g.S[c] = 0;
      h.down();
      pops++;
    }
    for (int k = 0; k < 4; k++) {
      if (!((jm >> k) & 1ull)) continue;
      const int rz = k == 2 ? iz - 1 : k == 3 ? iz + 1 : iz, rx = k == 0 ? ix - 1 : k == 1 ? ix + 1 : ix;
      const int r = rz * nx + rx;
      // a usable entry?
      const unsigned long long hm = __ballot(X->spec[lane].cell == r);
      bool use = false;
      double v = 0.0;
      if (hm) {
        const int e = __ffsll((long long)hm) - 1;
        const int ev = X->spec[e].ver;
        const double ev_val = X->spec[e].val;
        bool clash = mver - ev > kXLog || ev_val == -1.0;
        for (int q = ev + lane; !clash && q < mver; q += 64) {
          const int m = X->logc[q & (kXLog - 1)];
          const int mz = m / nx, mx = m - mz * nx;
          const int dz = abs(mz - rz), dx = abs(mx - rx);
          clash = (dz + dx >= 1) && ((dz + dx <= 1) || (dz == 2 && dx == 0) || (dx == 2 && dz == 0) ||
                                     (dz == 1 && dx == 1));
        }
        use = __ballot(clash) == 0ull;
        v = ev_val;
        if (!use && ev_val != -1.0 && mver - ev <= kXLog) {
          // a stencil node changed: the entry still stands if update()'s stencil stage is unchanged
          int same = 0;
          if (lane == 0) {
            NbField nq;
            nq.load(g.T, g.S, nz, nx, rz, rx);
            same = update_nb_select(nq, rz, rx, nz, nx).same(X->spec[e].sel) ? 1 : 0;
          }
          use = __shfl(same, 0) != 0;
        }
      }
      if (!use) {  // one pass: this relaxation on lane 0, guesses of the next pops' on the others
        int cz = rz, cx = rx;
        bool cand = true;
        if (lane > 0) {
          const int p = 1 + ((lane - 1) >> 2), d = (lane - 1) & 3;
          const int hc = X->cell[p];
          const int hz = hc / nx, hx = hc - hz * nx;
          cz = hz + (d == 2 ? -1 : d == 3 ? 1 : 0);
          cx = hx + (d == 0 ? -1 : d == 1 ? 1 : 0);
          cand = hc >= 0 && hc < nz * nx && cz >= 0 && cz < nz && cx >= 0 && cx < nx;
        }
        NbField nb;
        CellMat cm;
        if (cand) {
          cm = cell_mat(M, g.mv, cz, cx);
          nb.load(g.T, g.S, nz, nx, cz, cx);
        }
        if (cand && lane > 0) cand = g.S[cz * nx + cx] != 0;  // not known (a guess)
        if (cand) {
          const UpdSel sel = update_nb_select(nb, cz, cx, nz, nx);
          const double val = update_nb_finish(M, cm, cz, cx, g.dnx, sel);
          X->spec[lane].cell = cz * nx + cx;
          X->spec[lane].ver = mver;
          X->spec[lane].val = val;
          X->spec[lane].sel = sel;
          if (lane == 0) v = val;
        } else {
          X->spec[lane].cell = -1;
        }
        npass++;
      }
      if (lane == 0) {
        if (v == -1.0) {
          GField F{g.T, g.S, nz, nx};
          v = fouds18(F, M, cell_mat(M, g.mv, rz, rx), rz, rx, g.dnx, g.dnz, nx, nz, mat_slo(M, g.mv, rz, rx));
        }
        if (box) box->add(rz, rx);
        g.T[r] = v;
        if (stk[k] == -1) h.add(r, v, true);
        else h.upd(r, g.S[r], v);  // its heap index now (earlier sift-ups may have moved it)
        if (h.ndup) h.sync(r, v);
        X->logc[mver & (kXLog - 1)] = r;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the commit before any later load
      }
      mver++;
    }
  }
  if (prof && lane == 0) {  // diagnostics: relaxations, evaluation passes (BandSrc::sub, read by band_profile)
    prof[0] += mver;
    prof[1] += npass;
  }
  return pops;
}

// hand-over of every 3rd node of a stage grid into the next grid, in row-major order (:2391-2425,
// :2725-2759): ttn copied, known nodes stay known, "outer" known nodes and close nodes -> heap
AF_DEV void xhandover(XHeap& h, const XGrid& s, int isz_s, int isx_s, const XGrid& d, int isz_d, int isx_d,
                      XBox* box = nullptr) {
  for (int i = 0; i < s.nz + 1; i += 3) {
    for (int j = 0; j < s.nx + 1; j += 3) {
      const int pz = isz_d + (i - isz_s) / 3, px = isx_d + (j - isx_s) / 3;
      const int dc = pz * d.nx + px;
      d.T[dc] = s.T[i * s.nx + j];
      if (box) box->add(pz, px);
      const int st = s.S[i * s.nx + j];
      if (st == 0) {
        d.S[dc] = 0;
        bool outer = false;
        if (i - 3 >= 0) { if (s.S[(i - 3) * s.nx + j] == -1) outer = true; } else outer = true;
        if (i + 3 <= s.nz - 1) { if (s.S[(i + 3) * s.nx + j] == -1) outer = true; } else outer = true;
        if (j - 3 >= 0) { if (s.S[i * s.nx + j - 3] == -1) outer = true; } else outer = true;
        if (j + 3 <= s.nx - 1) { if (s.S[i * s.nx + j + 3] == -1) outer = true; } else outer = true;
        if (outer) h.add(dc);
      }
      if (st > 0) h.add(dc);
    }
  }
}

AF_DEV void xclear(double* T, int* S, int n) {
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    T[k] = __builtin_nan("");  // far (fields.h: far cells of HBM grids hold NaN)
    S[k] = -1;
  }
}

__global__ __launch_bounds__(64) void fmm_exact_kernel(BandParams P) {
  __shared__ XLds lds;
  const int src = blockIdx.x;
  crm::lds_init();
  if (src >= P.nsrc) return;
  BandSrc* B = P.src + src;
  const int lane = threadIdx.x;
  const DevModel& M = P.M;
  const int sg = P.sg, sgside = (sg - 1) / 2;
  const long isx = (long)sg * (long)rint((P.scx[src] - P.gox) / P.dnx);
  const long isz = (long)sg * (long)rint((P.scz[src] - P.goz) / P.dnz);
  const int nnz = P.nz, nnx = P.nx;
  int err = 0;
  XGrid prev{nullptr, nullptr, 0, 0, MatView{}, 0, 0};
  int pisz = 0, pisx = 0;
  const int scales[2] = {9, 3};
  const int size1 = 2 * sg + (sg - 1) / 2, size2 = size1 + 3 * sg;
  for (int stg = 0; stg < 2 && !err; stg++) {
    const int scale = scales[stg], size = stg == 0 ? size1 : size2;
    const int left = (int)max(0L, isx - size), right = (int)min((long)nnx - 1, isx + size);
    const int bottom = (int)max(0L, isz - size), top = (int)min((long)nnz - 1, isz + size);
    XGrid g;
    g.nz = scale * (top - bottom) + 1;
    g.nx = scale * (right - left) + 1;
    if ((long)g.nz * g.nx > P.capS) {
      err = 4;
      break;
    }
    g.T = gptr(B->Ts[stg]);
    g.S = gptr(B->Ss[stg]);
    g.mv = MatView{scale, (scale - 1) / 2, bottom, scale, (scale - 1) / 2, left, sg, sgside, 0, 0, 1};
    g.dnx = g.dnz = P.dnx / scale;
    const int isx_s = scale * (int)(isx - left), isz_s = scale * (int)(isz - bottom);
    xclear(g.T, g.S, g.nz * g.nx);
    __syncthreads();
    XHeap h{&lds, g.S, g.T, 0, 0};
    if (stg == 0) {
      // straight rays (:2223-2267; veln + angle, SURVEY B-D5), material of the source's fine cell
      const int side1 = (9 - 1) / 2 + 9 * ((sg - 1) / 2);
      const MatView fine{sg, sgside, 0, sg, sgside, 0, 1, 0, 0, 0, 1};
      const CellMat cs = cell_mat(M, fine, (int)isz, (int)isx);
      const int w = 2 * side1 + 1;
      for (int k = lane; k < w * w; k += blockDim.x) {
        const int i = k / w - side1, j = k % w - side1;
        if (0 <= isz_s + i && isz_s + i <= g.nz - 1 && 0 <= isx_s + j && isx_s + j <= g.nx - 1) {
          double angle = (j == 0) ? 90.0 : AF_ATAN((double)i / (double)j) * kRad2Deg;
          double eff = pymod(cs.veln + angle, 180);
          double velocity = (cs.velpn != 0 || cs.stif == nullptr) ? table_vel(M.gtab, M.ncol, eff, cs.velpn, cs.vm)
                                                                  : christoffel_group(cs.stif, eff, cs.vm);
          double length = g.dnx * sqrt((double)(i * i + j * j));
          g.T[(isz_s + i) * g.nx + isx_s + j] = length / velocity;
          g.S[(isz_s + i) * g.nx + isx_s + j] = 0;
        }
      }
      __syncthreads();
      if (lane == 0) {
        // window edges -> heap in the reference's order (:2277-2288)
        const int s1 = side1;
        if (isz_s - s1 >= 0)
          for (int i = max(0, isx_s - s1); i <= min(g.nx - 1, isx_s + s1); i++) h.add((isz_s - s1) * g.nx + i);
        if (isz_s + s1 <= g.nz - 1)
          for (int i = max(0, isx_s - s1); i <= min(g.nx - 1, isx_s + s1); i++) h.add((isz_s + s1) * g.nx + i);
        if (isx_s - s1 >= 0)
          for (int i = max(0, isz_s - s1); i <= min(g.nz - 1, isz_s + s1); i++) h.add(i * g.nx + isx_s - s1);
        if (isx_s + s1 <= g.nx - 1)
          for (int i = max(0, isz_s - s1); i <= min(g.nz - 1, isz_s + s1); i++) h.add(i * g.nx + isx_s + s1);
      }
    } else if (lane == 0) {
      xhandover(h, prev, pisz, pisx, g, isz_s, isx_s);
    }
    if (lane == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // grid stores before the walk's loads
    {
      const long long pops = xloop_spec(h, M, g, true, isx_s, isz_s, scale * size, 0.0, nullptr, lane, B->sub);
      if (lane == 0) {
        B->steps[stg] = pops;
        err = h.err;
      }
    }
    err = __shfl(err, 0);
    __syncthreads();
    prev = g;
    pisz = isz_s;
    pisx = isx_s;
  }
  // fine main grid (memset by the host: T 0, S -1): hand-over, then the exact prefix
  {
    XGrid g;
    g.T = gptr(B->T);
    g.S = gptr(B->S);
    g.nz = nnz;
    g.nx = nnx;
    g.mv = MatView{sg, sgside, 0, sg, sgside, 0, 1, 0, 0, 0, 1};
    g.dnx = P.dnx;  // the coarse spacing on the fine grid (:2790; field divided by sg at the end)
    g.dnz = P.dnz;
    XHeap h{&lds, g.S, g.T, 0, 0};
    XBox box;  // what the K-member band kernel copies into its edge buffers
    if (!err && lane == 0) {
      xhandover(h, prev, pisz, pisx, g, (int)isz, (int)isx, &box);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (!err) {
      const long long pops = xloop_spec(h, M, g, false, 0, 0, 0, P.tstop, &box, lane, B->sub);
      if (lane == 0) B->steps[2] = pops;
    }
    if (lane == 0) {
      int nl = 0;
      if (!err) {
        for (int q = 0; q < 4; q++) B->bbox[q] = box.b[q];
        err = h.err;
        // heap -> band close list (statuses: heap index > 0 -> close 1)
        for (int k = 1; k <= h.ntr && k <= P.capL; k++) {
          const int c = lds.cell[k];
          B->S[c] = k;  // close: 1 + close-list slot
          B->Lin[k - 1] = c;
        }
        nl = h.ntr;
        if (nl > P.capL) err = 2;
      }
      B->nl0 = nl;
      B->err = err;
    }
  }
}

}  // namespace af

extern "C" hipError_t af_launch_exact(const af::BandParams* P, hipStream_t stream) {
  hipLaunchKernelGGL(af::fmm_exact_kernel, dim3(P->nsrc), dim3(64), 0, stream, *P);
  return hipGetLastError();
}
