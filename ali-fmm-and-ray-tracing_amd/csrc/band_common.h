// band_common.h — helpers of the band-synchronous FMM kernel (fmm_band_k.hip: one source over
// K = 1..16 workgroups) and the exact-order kernel (fmm_exact.hip).
#pragma once
#include "kernels.h"

namespace af {

template <class T, int CAP>
struct HList {
  T* l;  // LDS head
  T* g;  // global array (same indexing)
  AF_DEV T get(int i) const { return i < CAP ? l[i] : gld(g + i); }
  // callers that checked (uniformly) that every index is below CAP: plain LDS accesses that the
  // compiler can batch (get/put branch per access to the global spill)
  AF_DEV T lds(int i) const { return l[i]; }
  AF_DEV void put_lds(int i, T v) const { l[i] = v; }
  AF_DEV void put(int i, T v) const {
    if (i < CAP) l[i] = v;
    else gst(g + i, v);
  }
};

AF_DEV int lane_id() { return threadIdx.x & 63; }


// Uniform double kept in (and re-read from) scalar registers: the compiler cannot hoist
// expressions derived from it above this point.  The persistent band kernels launder their
// step-invariant doubles per phase so that derived constants are not kept live (and spilled to
// scratch: a memory round trip per reload) across the step loop.
AF_DEV double launder_u(double v) {
  const long long b = __double_as_longlong(v);
  int lo = __builtin_amdgcn_readfirstlane((int)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  asm volatile("" : "+s"(lo), "+s"(hi));
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// append with one LDS atomic per wave; returns the slot or -1 (pred false / overflow)
AF_DEV int wave_push(int* counter, bool pred, int cap, int* err) {
  unsigned long long m = __ballot(pred);
  if (m == 0) return -1;
  int lane = lane_id();
  int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, __popcll(m));
  base = bcast(base, leader);
  int off = __popcll(m & ((1ull << lane) - 1ull));
  if (!pred) return -1;
  int slot = base + off;
  if (slot >= cap) {
    *err = 2;
    return -1;
  }
  return slot;
}

// wave_push onto two counters with the same predicate (both LDS atomics in flight together)
AF_DEV void wave_push2(int* c1, int* c2, bool pred, int cap, int* err, int& s1, int& s2) {
  s1 = s2 = -1;
  unsigned long long m = __ballot(pred);
  if (m == 0) return;
  int lane = lane_id();
  int leader = __ffsll((long long)m) - 1;
  int b1 = 0, b2 = 0;
  if (lane == leader) {
    b1 = atomicAdd(c1, __popcll(m));
    b2 = atomicAdd(c2, __popcll(m));
  }
  b1 = bcast(b1, leader);
  b2 = bcast(b2, leader);
  if (!pred) return;
  int off = __popcll(m & ((1ull << lane) - 1ull));
  s1 = b1 + off;
  s2 = b2 + off;
  if (s1 >= cap || s2 >= cap) {
    *err = 2;
    s1 = s2 = -1;
  }
}

AF_DEV double wave_min(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  return v;
}

// Wave reductions by DPP moves inside each row of 16 lanes (quad xor 1, quad xor 2, half-row
// mirror, row mirror) and v_readlane of the four rows: no LDS round trips (a __shfl_xor ladder is
// six ds_bpermute round trips, twelve for a double).  EVERY lane of the wave must be active.
template <int CTRL>
AF_DEV int dppm_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
AF_DEV double dppm_d(double v) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)dppm_i<CTRL>((int)b), hi = (unsigned)dppm_i<CTRL>((int)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
AF_DEV double rdlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
AF_DEV double wave_min_full(double v) {
  v = fmin(v, dppm_d<0xB1>(v));
  v = fmin(v, dppm_d<0x4E>(v));
  v = fmin(v, dppm_d<0x141>(v));
  v = fmin(v, dppm_d<0x140>(v));
  return fmin(fmin(rdlane_d(v, 0), rdlane_d(v, 16)), fmin(rdlane_d(v, 32), rdlane_d(v, 48)));
}
AF_DEV int wave_sum_full(int v) {
  v += dppm_i<0xB1>(v);
  v += dppm_i<0x4E>(v);
  v += dppm_i<0x141>(v);
  v += dppm_i<0x140>(v);
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}
AF_DEV int wave_or_full(int v) {
  v |= dppm_i<0xB1>(v);
  v |= dppm_i<0x4E>(v);
  v |= dppm_i<0x141>(v);
  v |= dppm_i<0x140>(v);
  return __builtin_amdgcn_readlane(v, 0) | __builtin_amdgcn_readlane(v, 16) | __builtin_amdgcn_readlane(v, 32) |
         __builtin_amdgcn_readlane(v, 48);
}

// Lists hold cells as packed (z << 16 | x) keys (grids are < 32768 per side): no integer
// divisions on the hot path; the flat index z * nx + x is formed where memory is addressed.
AF_DEV int pk(int z, int x) { return (z << 16) | x; }
AF_DEV int pkz(int k) { return k >> 16; }
AF_DEV int pkx(int k) { return k & 0xffff; }
AF_DEV int pk_flat(int k, int nx) { return pkz(k) * nx + pkx(k); }

// neighbour d (0 -x, 1 +x, 2 -z, 3 +z) of packed cell c, or -1 outside the grid
AF_DEV int nb_cell(int c, int d, int nz, int nx) {
  const int z = pkz(c) + (d == 2 ? -1 : d == 3 ? 1 : 0);
  const int x = pkx(c) + (d == 0 ? -1 : d == 1 ? 1 : 0);
  return (z < 0 || z >= nz || x < 0 || x >= nx) ? -1 : pk(z, x);
}

// exclusive prefix sum over the wave's lanes, and the wave total: DPP row shifts (1, 2, 4, 8)
// then row broadcasts 15 / 31 (a disabled source lane contributes the 0 "old" value); EVERY
// lane of the wave must be active
AF_DEV int wave_excl_scan(int v, int& total) {
  int inc = v;
  inc += __builtin_amdgcn_update_dpp(0, inc, 0x111, 0xf, 0xf, false);  // row_shr:1
  inc += __builtin_amdgcn_update_dpp(0, inc, 0x112, 0xf, 0xf, false);  // row_shr:2
  inc += __builtin_amdgcn_update_dpp(0, inc, 0x114, 0xf, 0xf, false);  // row_shr:4
  inc += __builtin_amdgcn_update_dpp(0, inc, 0x118, 0xf, 0xf, false);  // row_shr:8
  inc += __builtin_amdgcn_update_dpp(0, inc, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  inc += __builtin_amdgcn_update_dpp(0, inc, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  total = bcast(inc, 63);
  return inc - v;
}

// Column-stripe ownership of the K-member band kernel (fmm_band_k.hip): stripe s = x >> wlog
// (W = 2^wlog columns, W >= 8) belongs to member s mod K (K = 1..16; the modulo by a multiply with
// kmagic = ceil(2^16 / K), exact for every stripe index below 4096).  EDGE cells lie
// within 2 columns of a stripe boundary (another member's 12-point / 5x5 stencils read them; they
// are mirrored in the edge buffers: 4 columns per stripe, column-major, eidx), RIM cells next to
// one (their 4-neighbour across the boundary belongs to another member).  K = 1: no edges, no rims.
struct KGeom {
  int K, wlog, nz, nx, kmagic;
  AF_DEV int owner(int x) const {
    const int st = x >> wlog;
    return st - K * ((st * kmagic) >> 16);
  }
  AF_DEV bool edge(int x) const {
    const int r = x & ((1 << wlog) - 1);
    return K > 1 && (r < 2 || r >= (1 << wlog) - 2);
  }
  AF_DEV bool rim(int x) const {
    const int r = x & ((1 << wlog) - 1);
    return K > 1 && ((r == 0 && x > 0) || (r == (1 << wlog) - 1 && x < nx - 1));
  }
  // edge-buffer column of an edge column x, and the entry of cell (z, x)
  AF_DEV int ecol(int x) const {
    const int r = x & ((1 << wlog) - 1);
    return ((x >> wlog) << 2) + (r < 2 ? r : r - ((1 << wlog) - 4));
  }
  AF_DEV int eidx(int z, int x) const { return ecol(x) * nz + z; }
  // column x + dx (|dx| <= 2) of an own cell at column x lies in another member's stripe
  AF_DEV bool other(int x, int dx) const {
    const int r = (x & ((1 << wlog) - 1)) + dx;
    return K > 1 && (r < 0 || r >= (1 << wlog)) && x + dx >= 0 && x + dx < nx;
  }
};

struct RunCfg {
  int nz, nx;
  double dnx, dnz;  // update() spacing and fouds18 dnz
  MatView mv;
  double delta, t0;
  double delta_far, tfar;  // band width far from the source (tfar 0: off)
};

// material of main-grid cell (z, x): LDSMAT = one id load + the LDS record; else four arrays.
// IDENT: the main grid is the model grid (subgrid 1): no view arithmetic (its four integer
// divisions), and the ids from the bricked copy when there is one
template <bool LDSMAT, bool IDENT = false>
AF_DEV CellMat band_mat(const DevModel& M, const MatRec* mat, const double* stab, const MatView& v, int z, int x) {
  if (!LDSMAT) return cell_mat(M, v, z, x);
  int id;
  if (IDENT && M.mid8b) {
    id = (int)gld(M.mid8b + ((((long)(z >> 3) * M.mid8b_pitch + (x >> 4)) << 7) | ((z & 7) << 4) | (x & 15)));
  } else {
    const long i = IDENT ? (long)z * M.nx0 + x : mv_cell(M, v, z, x);
    id = M.mid8 ? (int)gld(M.mid8 + i) : gld(M.mid + i);
  }
  const MatRec m = mat[id];
  CellMat r;
  r.velpn = m.velpn;
  r.veln = v.quant ? (double)(int)m.veln : m.veln;
  r.vm = v.quant ? (double)(float)m.vm : m.vm;
  r.stif = m.sidx >= 0 ? stab + 5 * m.sidx : nullptr;
  return r;
}


}  // namespace af
