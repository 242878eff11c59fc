// device_common.h — shared gfx950 device code for the ALI-FMM travel-time-field solver.
//
// The local operators below are the reference's arithmetic (Anis_TTF_rays.py, cited per
// function) in double precision, operation order preserved and compiled with
// -ffp-contract=off, so that a cell evaluated on the same neighbourhood matches the CPU
// oracle to the last bit except where the trigonometric functions differ from glibc's.
// AF_CRMATH (default 1): atan / sin / cos / tan are cr_math.h's correctly rounded ones (glibc's
// results on all but ~0.1 % of arguments, where glibc itself is off by just over half an ulp);
// 0: ocml's (~1 % of results an ulp away).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef AF_CRMATH
#define AF_CRMATH 1
#endif
#include "cr_math.h"
#if AF_CRMATH
#define AF_ATAN crm::atan
#define AF_SIN crm::sin
#define AF_COS crm::cos
#define AF_TAN crm::tan
#define AF_SINCOS crm::sincos
#else
#define AF_ATAN atan
#define AF_SIN sin
#define AF_COS cos
#define AF_TAN tan
#define AF_SINCOS sincos
#endif

#define AF_DEV __device__ __forceinline__

namespace af {

// Global-memory accesses through pointers the compiler cannot prove global (pointers stored in
// device-side structs, e.g. BandSrc) would otherwise compile to flat_* instructions, whose
// completion also counts on lgkmcnt and so serialises them against every LDS access.
#define AF_GLOBAL __attribute__((address_space(1)))
template <class T>
AF_DEV T gld(const T* p) {
  return *(const AF_GLOBAL T*)p;
}
template <class T>
AF_DEV void gst(T* p, T v) {
  *(AF_GLOBAL T*)p = v;
}
// the same pointer with its global address space made visible (an addrspace cast round trip):
// plain loads and stores through it compile to global_* instead of flat_*
template <class T>
AF_DEV T* gptr(T* p) {
  return (T*)(AF_GLOBAL T*)p;
}
AF_DEV int gatomic_max(int* p, int v) { return __atomic_fetch_max((AF_GLOBAL int*)p, v, __ATOMIC_RELAXED); }
// sc1 (L1-bypassing load, write-through store) accesses for data another CU writes or reads
// within the same launch (MI355X_MICROARCH.md "inter-workgroup visibility": sc1 stores, drained
// with vmcnt(0) before the signal, read back with sc1 loads after the signal)
template <class T>
AF_DEV T gld_sc1(const T* p) {
  return __hip_atomic_load((AF_GLOBAL T*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
AF_DEV void gst_sc1(T* p, T v) {
  __hip_atomic_store((AF_GLOBAL T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr double kDeg2Rad = M_PI / 180.0;
constexpr double kRad2Deg = 180.0 / M_PI;

// Python float '%' (CPython float_divmod; numba real_divmod_func_body).
// Fast paths for |a| < 2b (every call site: angles mod 180/90/pi) give the same bits as the
// generic fmod route: fmod(a, b) is exact, and a -/+ b is exact there by Sterbenz's lemma; the
// only rounding is the final '+ b' of negative remainders, which the reference performs too.
// value of lane l (wave-uniform l) for every lane: v_readlane into a scalar register, no LDS round
// trip (a __shfl from one lane is a ds_bpermute: an LDS round trip in the wave's dependent chain)
AF_DEV int bcast(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
AF_DEV unsigned long long bcast64(unsigned long long v, int l) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}

AF_DEV double pymod(double a, double b) {
  if (b > 0) {
    if (a >= 0 && a < b) return a == 0 ? 0.0 : a;  // -0.0 -> +0.0 as copysign(0, b)
    if (a >= b && a < 2 * b) return a - b;
    if (a < 0 && a >= -b) return a + b;            // a == -b: fmod gives -0.0 -> +0.0, as here
    if (a < -b && a > -2 * b) return (a + b) + b;
  }
  double m = fmod(a, b);
  if (m != 0.0) {
    if ((b < 0) != (m < 0)) m += b;
  } else {
    m = copysign(0.0, b);
  }
  return m;
}
// round(): half-even (numba lowers to llvm.rint).
AF_DEV long pyround(double x) { return (long)rint(x); }
// the same for values known to fit in int (grid coordinates): two instructions instead of the
// 64-bit conversion's sequence
AF_DEV int pyround_i(double x) { return (int)rint(x); }

// ---------------------------------------------------------------------------------------------
// Distinct per-cell material (veln, vel_map, velpn, stiffness row): the band kernel stages the
// table in LDS and reads one 4-byte id per cell instead of four arrays.
struct MatRec {
  double veln, vm;
  int velpn, sidx;  // sidx -1: stif_den is None
};

// Model resident in HBM (uploaded once per set_model, shared by every source on the GPU).
struct DevModel {
  int nz0, nx0;          // coarse grid
  const double* veln;    // orientation [deg]
  const int* velpn;      // material column (0 = stiffness)
  const double* vm;      // velocity scale
  const int* sidx;       // stiffness row index per cell, or nullptr when stif_den is None
  const double* stab;    // unique stiffness rows [n][5] (exact int64 values as doubles)
  int nstab;             // number of unique stiffness rows
  const double* gtab;    // group velocity table (361, ncol)
  const double* ptab;    // phase velocity table (361, ncol)
  int ncol;
  const int* mid;        // material id per cell (into mtab), or nullptr when there are too many
  const unsigned char* mid8;  // the same ids as bytes when nmat <= 256, else nullptr
  const unsigned char* mid8b; // mid8 in 8 x 16 bricks (one 128-byte line each; pitch mid8b_pitch
  int mid8b_pitch;            // bricks per brick row), or nullptr: the band kernel's subgrid-1 view
  const MatRec* mtab;
  int nmat;
  const double* mslo;     // per material and MatView::quant: fouds18_A()'s 4 slownesses [nmat][2][4], or nullptr
};

// Logical grid -> coarse cell: f = lo1 + (a + side1)/s1 ; c = lo2 + (f + side2)/s2
// (finer_grid_n nearest-neighbour refinement, :26-56; windows :1516-1529, :2191-2204).
struct MatView {
  int s1z, side1z, lo1z, s1x, side1x, lo1x;
  int s2, side2, lo2z, lo2x;
  int quant;  // finer_grid_n quantisation: veln -> int32 (trunc), vel_map -> float32
};

AF_DEV long mv_cell(const DevModel& M, const MatView& v, int iz, int ix) {
  int fz = v.lo1z + (iz + v.side1z) / v.s1z;
  int fx = v.lo1x + (ix + v.side1x) / v.s1x;
  int cz = v.lo2z + (fz + v.side2) / v.s2;
  int cx = v.lo2x + (fx + v.side2) / v.s2;
  return (long)cz * M.nx0 + cx;
}

// fouds18_A()'s four slownesses of cell (iz, ix)'s material under view v (DevModel::mslo,
// precomputed per material on the device), or nullptr when the model has no material table
AF_DEV const double* mat_slo(const DevModel& M, const MatView& v, int iz, int ix) {
  if (!M.mid || !M.mslo) return nullptr;
  return M.mslo + 8 * (long)gld(M.mid + mv_cell(M, v, iz, ix)) + 4 * (v.quant ? 1 : 0);
}

struct CellMat {
  double veln, vm;
  int velpn;
  const double* stif;  // nullptr => None
};

AF_DEV CellMat cell_mat(const DevModel& M, const MatView& v, int iz, int ix) {
  long c = mv_cell(M, v, iz, ix);
  CellMat r;
  double a = gld(M.veln + c);
  double b = gld(M.vm + c);
  r.veln = v.quant ? (double)(int)a : a;
  r.vm = v.quant ? (double)(float)b : b;
  r.velpn = gld(M.velpn + c);
  r.stif = M.sidx ? M.stab + 5 * (long)gld(M.sidx + c) : nullptr;
  return r;
}

// Table lookup, linear in 1-degree bins (:288-291, :1372-1375, :2951-2954).
AF_DEV double table_vel(const double* tab, int ncol, double eff, int col, double vm) {
  long a1 = (long)floor(eff);
  long a2 = (a1 + 1) % 180;
  double rem = eff - (double)a1;
  return vm * ((1 - rem) * tab[a1 * ncol + col] + rem * tab[a2 * ncol + col]);
}

// Closed-form 2D orthotropic Christoffel GROUP velocity (:294-315, group_vel :3542-3558).
// s[] holds exact integers, so double arithmetic reproduces the reference's int64 sums/products.
AF_DEV double christoffel_group(const double* s, double eff, double vm) {
  double sigma = s[4];
  double e90 = pymod(eff, 90);
  if (e90 < 0.01 || e90 > 90 - 0.01) {
    double lam = (fabs(pymod(eff, 180) - 90) < 1) ? s[2] : s[0];
    return 1000 * vm * sqrt(lam / sigma);
  }
  double c22 = s[0], c23 = s[1], c33 = s[2], c44 = s[3];
  double tan_ang = AF_TAN(eff * kDeg2Rad);
  double A = c22 + c33 - 2 * c44;
  double B = (c23 + c44) * (tan_ang - 1 / tan_ang);
  double C = c22 - c33;
  double disc = B * B + A * A - C * C;
  double pa;
  if (eff < 90)
    pa = pymod(AF_ATAN((-B - sqrt(disc)) / (C - A)), M_PI);
  else
    pa = pymod(AF_ATAN((-B + sqrt(disc)) / (C - A)), M_PI);
  double s2, c2;  // sin and cos of 2 pa from one reduction
  AF_SINCOS(2 * pa, &s2, &c2);
  double lam = 0.5 * (c2 * (c22 - c44) + s2 * (c23 + c44) * tan_ang + c22 + c44);
  return 1000 * vm * sqrt(lam / sigma) / AF_COS(eff * kDeg2Rad - pa);
}

// Christoffel PHASE velocity (update() :1400-1406).
AF_DEV double christoffel_phase(const double* s, double eff, double vm) {
  double sa, ca;
  AF_SINCOS(eff * kDeg2Rad, &sa, &ca);
  double A = ca * ca * s[0] + sa * sa * s[3];
  double B = ca * sa * (s[1] + s[3]);
  double C = ca * ca * s[3] + sa * sa * s[2];
  return 1000 * vm * sqrt((A + C + sqrt((A - C) * (A - C) + 4 * (B * B))) / (2 * s[4]));
}

// group velocity with the selector 'velpn != 0 or stif_den == None' (:287, :2950); gtab: the
// group-velocity table (M.gtab or a copy in LDS)
AF_DEV double group_vel_cell(const DevModel& M, const CellMat& c, double eff, const double* gtab) {
  if (c.velpn != 0 || c.stif == nullptr) return table_vel(gtab, M.ncol, eff, c.velpn, c.vm);
  return christoffel_group(c.stif, eff, c.vm);
}
AF_DEV double group_vel_cell(const DevModel& M, const CellMat& c, double eff) {
  return group_vel_cell(M, c, eff, M.gtab);
}

// Material sources of time_between_points() on the coarse grid (identity view): the model
// arrays in HBM, or the material-id bytes plus the distinct records, stiffness rows and group
// table staged in LDS by the kernel (the same values: the records are the model's).
struct MatGlobal {
  const DevModel& M;
  AF_DEV int id(int z, int x) const { return M.mid ? gld(M.mid + (long)z * M.nx0 + x) : -1; }
  AF_DEV CellMat cm(int, int z, int x) const {
    const MatView ident{1, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0};
    return cell_mat(M, ident, z, x);
  }
  AF_DEV const double* gtab() const { return M.gtab; }
};
struct MatLds {
  const DevModel& M;
  const MatRec* mat;
  const double* stab;
  const double* gt;
  AF_DEV int id(int z, int x) const {
#ifdef AF_RAY_DIAG_NOID  // diagnostic build only (wrong rays): the cost of the material-id loads
    return 0;
#endif
    const long c = (long)z * M.nx0 + x;
    return M.mid8 ? (int)gld(M.mid8 + c) : gld(M.mid + c);
  }
  AF_DEV CellMat cm(int id, int, int) const {
    const MatRec m = mat[id];
    return CellMat{m.veln, m.vm, m.velpn, m.sidx >= 0 ? stab + 5 * m.sidx : nullptr};
  }
  AF_DEV const double* gtab() const { return gt; }
};

// wavefront_angle_dist :1413-1460
template <class I>
AF_DEV void wad(I ix, I iz, I x1, I x2, I x3, I z1, I z2, I z3, double y1, double y2, double y3, double& angle,
                double& dist) {
  double a;
  if (y3 != y1) {
    a = (y2 - y1) / (y3 - y1);
  } else {
    angle = 0.0;
    dist = -1.0;
    return;
  }
  double xpos = (1 - a) * (double)x1 + a * (double)x3;
  double zpos = (1 - a) * (double)z1 + a * (double)z3;
  double dx = (double)x2 - xpos;
  double dz = (double)z2 - zpos;
  if (dx == 0)
    angle = 0.0;
  else
    angle = pymod(AF_ATAN(dz / dx) * kRad2Deg + 90, 180);
  dist = fabs(dz * (double)(x2 - ix) - dx * (double)(z2 - iz)) / sqrt(dx * dx + dz * dz);
}

// time_between_points :2835-2989 (coarse material, numba negative-index wrap)
// The walk over the segment's pieces (crossings of the half-integer cell edges): the geometry of
// piece k does not depend on the material, only the slowness does.
struct TbpWalk {
  double start_x, start_y, end_x, end_y, mm, cc;
  double next_x, next_y, prev_x, prev_y;
  int dir_x, dir_y;
  bool fin_x, fin_y;
  // the segment (x1, y1) -> (x2, y2) in subgrid-sg coordinates; *angle: its direction [deg]
  AF_DEV void setup(double x1, double x2, double y1, double y2, int sg, double& angle) {
    if (sg != 1) {  // (x / 1.0 is x)
      x1 = x1 / (double)sg;
      x2 = x2 / (double)sg;
      y1 = y1 / (double)sg;
      y2 = y2 / (double)sg;
    }
    start_x = x1;
    end_x = x2;
    start_y = y1;
    end_y = y2;
    angle = (x1 == x2) ? 0.0 : AF_ATAN((y2 - y1) / (x2 - x1)) * kRad2Deg;
    mm = 0;
    cc = 0;
    if (end_x != start_x) {
      mm = (end_y - start_y) / (end_x - start_x);
      cc = start_y - mm * start_x;
    }
    dir_x = (start_x < end_x) ? 1 : -1;
    dir_y = (start_y < end_y) ? 1 : -1;
  }
  AF_DEV void begin() {
    fin_x = fin_y = false;
    next_x = rint(start_x) + dir_x * 0.5;  // (double)pyround(x) is rint(x)
    next_y = rint(start_y) + dir_y * 0.5;
    prev_x = start_x;
    prev_y = start_y;
  }
  AF_DEV bool done() const { return fin_x && fin_y; }
  // the next piece's end point (nxv, nyv); the piece runs from (prev_x, prev_y)
  AF_DEV void piece(double& nxv, double& nyv) {
    if (((next_x > end_x && dir_x == 1) || (next_x < end_x && dir_x == -1)) && !fin_x) {
      fin_x = true;
      next_x = end_x;
    }
    if (((next_y > end_y && dir_y == 1) || (next_y < end_y && dir_y == -1)) && !fin_y) {
      fin_y = true;
      next_y = end_y;
    }
    if (end_x == start_x) {
      nxv = start_x;
      nyv = next_y;
      next_y += dir_y;
    } else {
      double next_x_yval = mm * next_x + cc;
      if (mm != 0) {
        double next_y_xval = (next_y - cc) / mm;
        double d1x = start_x - next_x, d1y = start_y - next_x_yval;
        double d2x = start_x - next_y_xval, d2y = start_y - next_y;
        if (d1x * d1x + d1y * d1y < d2x * d2x + d2y * d2y) {
          nxv = next_x;
          nyv = next_x_yval;
          next_x += dir_x;
        } else {
          nxv = next_y_xval;
          nyv = next_y;
          next_y += dir_y;
        }
      } else {
        nxv = next_x;
        nyv = next_x_yval;
        next_x += dir_x;
      }
    }
  }
  // the piece's coarse cell (midpoint, rounded; negative indices wrap like numba's)
  AF_DEV void cell(const DevModel& M, double nxv, double nyv, int& y_pos, int& x_pos) const {
    x_pos = pyround_i((prev_x + nxv) / 2);
    y_pos = pyround_i((prev_y + nyv) / 2);
    if (x_pos < 0) x_pos += M.nx0;
    if (y_pos < 0) y_pos += M.nz0;
  }
  // the piece's length [m] and its time at slowness slown (time_between_points' summand)
  AF_DEV double piece_dist(double nxv, double nyv, double dnx) const {
    double ddx = prev_x - nxv, ddy = prev_y - nyv;
    return dnx * sqrt(ddx * ddx + ddy * ddy);
  }
  AF_DEV double piece_time(double nxv, double nyv, double dnx, double slown) const {
    return piece_dist(nxv, nyv, dnx) * slown;
  }
};

// slowness of material record cm along a segment at angle [deg]
template <class MS>
AF_DEV double tbp_slowness(const DevModel& M, const MS& ms, const CellMat& cm, double angle) {
  double eff = pymod(cm.veln - angle, 180);
  double velocity = group_vel_cell(M, cm, eff, ms.gtab());
  return 1.0 / velocity;
}

template <class MS>
AF_DEV double tbp(const DevModel& M, const MS& ms, double x1, double x2, double y1, double y2, double dnx, int sg) {
  double section_time = 0.0;
  TbpWalk w;
  double angle;
  w.setup(x1, x2, y1, y2, sg, angle);
  w.begin();
  int last_id = -1;
  double slown = 0.0;
  while (!w.done()) {
    double nxv, nyv;
    w.piece(nxv, nyv);
    int y_pos, x_pos;
    w.cell(M, nxv, nyv, y_pos, x_pos);
    // the slowness depends on the cell only through its material record (the angle is fixed for
    // the segment), so consecutive pieces in the same material reuse it: the same value, without
    // the group-velocity evaluation (the per-cell material id identifies the record exactly)
    const int id = ms.id(y_pos, x_pos);
    if (id < 0 || id != last_id) {
      slown = tbp_slowness(M, ms, ms.cm(id, y_pos, x_pos), angle);
      last_id = id;
    }
    section_time += w.piece_time(nxv, nyv, dnx, slown);
    w.prev_x = nxv;
    w.prev_y = nyv;
  }
  return section_time;
}
AF_DEV double tbp(const DevModel& M, double x1, double x2, double y1, double y2, double dnx, int sg) {
  return tbp(M, MatGlobal{M}, x1, x2, y1, y2, dnx, sg);
}

}  // namespace af
