// fields.h — global-memory field accessors for the local operators (update() / fouds18_A()).
#pragma once
#include "device_common.h"

namespace af {

// Far cells of the HBM grids hold NaN (kFarT) instead of the reference's 0 so that validity can
// be read from T alone (NbFieldT); every value read through an accessor maps NaN back to 0, the
// reference's ttn of a never-relaxed node.
AF_DEV double far0(double v) { return v == v ? v : 0.0; }

struct GField {
  const double* T;
  const int* S;
  int nz, nx;
  AF_DEV int st(long z, long x) const { return z >= nz ? -1 : gld(S + z * nx + x); }
  AF_DEV double tt(long z, long x) const { return z >= nz ? 0.0 : far0(gld(T + z * nx + x)); }
};

// GField with sc1 loads: a grid that another workgroup of the same launch also writes
struct GFieldSC1 {
  const double* T;
  const int* S;
  int nz, nx;
  AF_DEV int st(long z, long x) const { return z >= nz ? -1 : gld_sc1(S + z * nx + x); }
  AF_DEV double tt(long z, long x) const { return z >= nz ? 0.0 : far0(gld_sc1(T + z * nx + x)); }
};

// Register copy of the 12 cells update() reads around (iz, ix): (0,+-1) (+-1,0) (+-1,+-1) (0,+-2)
// (+-2,0).  All 24 loads are issued together (one memory round trip instead of a chain of
// branch-dependent gathers).  Same values as GField: rows >= nz read status -1 / time 0 (the
// reference's padded stage-1 reads); other out-of-grid positions are never read by update().
struct NbField {
  long iz, ix;
  unsigned vm;  // bit k: status >= 0
  double t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, t11;
  AF_DEV static int slot(long dz, long dx) {
    return dz == 0 ? (dx == -2 ? 0 : dx == -1 ? 1 : dx == 1 ? 2 : 3)
         : dx == 0 ? (dz == -2 ? 4 : dz == -1 ? 5 : dz == 1 ? 6 : 7)
         : dz < 0 ? (dx < 0 ? 8 : 9) : (dx < 0 ? 10 : 11);
  }
  AF_DEV int st(long z, long x) const { return (vm >> slot(z - iz, x - ix)) & 1u ? 0 : -1; }
  AF_DEV double tt(long z, long x) const {
    const int k = slot(z - iz, x - ix);
    return k == 0 ? t0 : k == 1 ? t1 : k == 2 ? t2 : k == 3 ? t3 : k == 4 ? t4 : k == 5 ? t5 : k == 6 ? t6
         : k == 7 ? t7 : k == 8 ? t8 : k == 9 ? t9 : k == 10 ? t10 : t11;
  }
  // the cell at offset (dz, dx) now holds the valid value v (no-op outside the 12 positions)
  AF_DEV void patch(int dz, int dx, double v) {
    const int ad = abs(dz) + abs(dx);
    if (ad == 0 || ad > 2 || (dz != 0 && dx != 0 && (abs(dz) != 1 || abs(dx) != 1))) return;
    const int k = slot(dz, dx);
    vm |= 1u << k;
    t0 = k == 0 ? v : t0; t1 = k == 1 ? v : t1; t2 = k == 2 ? v : t2; t3 = k == 3 ? v : t3;
    t4 = k == 4 ? v : t4; t5 = k == 5 ? v : t5; t6 = k == 6 ? v : t6; t7 = k == 7 ? v : t7;
    t8 = k == 8 ? v : t8; t9 = k == 9 ? v : t9; t10 = k == 10 ? v : t10; t11 = k == 11 ? v : t11;
  }
  AF_DEV void load(const double* T, const int* S, int nz, int nx, int z, int x) {
    iz = z;
    ix = x;
    const long n = (long)nz * nx;
    long f[12];
    bool in[12];
    const int dz[12] = {0, 0, 0, 0, -2, -1, 1, 2, -1, -1, 1, 1};
    const int dx[12] = {-2, -1, 1, 2, 0, 0, 0, 0, -1, 1, -1, 1};
    int s[12];
    double t[12];
#pragma unroll
    for (int k = 0; k < 12; k++) {
      long c = (long)(z + dz[k]) * nx + (x + dx[k]);
      in[k] = z + dz[k] < nz;
      f[k] = c < 0 ? 0 : c >= n ? n - 1 : c;
    }
#pragma unroll
    for (int k = 0; k < 12; k++) {
      s[k] = gld(S + f[k]);
      t[k] = gld(T + f[k]);
    }
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < 12; k++) {
      if (in[k] && s[k] >= 0) m |= 1u << k;
      if (!in[k]) t[k] = 0.0;
    }
    vm = m;
    t0 = t[0]; t1 = t[1]; t2 = t[2]; t3 = t[3]; t4 = t[4]; t5 = t[5];
    t6 = t[6]; t7 = t[7]; t8 = t[8]; t9 = t[9]; t10 = t[10]; t11 = t[11];
  }
};

// As NbField, for update() (validity = nsts >= 0, i.e. known or close) on an HBM grid whose far
// cells hold NaN: 12 loads of T, no status loads.
struct NbFieldT {
  int iz, ix;
  unsigned vm;  // bit k: valid
  double t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, t11;
  AF_DEV int st(long z, long x) const { return (vm >> NbField::slot(z - iz, x - ix)) & 1u ? 0 : -1; }
  AF_DEV double tt(long z, long x) const {
    const int k = NbField::slot(z - iz, x - ix);
    return k == 0 ? t0 : k == 1 ? t1 : k == 2 ? t2 : k == 3 ? t3 : k == 4 ? t4 : k == 5 ? t5 : k == 6 ? t6
         : k == 7 ? t7 : k == 8 ? t8 : k == 9 ? t9 : k == 10 ? t10 : t11;
  }
  // 12 independent 8-byte loads at addresses clamped into the grid (no branches: a wavefront
  // issues them back to back); values at out-of-grid positions are never read by update() (it
  // bounds-checks first).  SC1: L1-bypassing loads, for cells another workgroup writes.
  template <bool SC1>
  AF_DEV void load_t(const double* T, int nz, int nx, int z, int x) {
    iz = z;
    ix = x;
    const int n = nz * nx;
    const int dz[12] = {0, 0, 0, 0, -2, -1, 1, 2, -1, -1, 1, 1};
    const int dx[12] = {-2, -1, 1, 2, 0, 0, 0, 0, -1, 1, -1, 1};
    const int p = z * nx + x;
    double t[12];
#pragma unroll
    for (int k = 0; k < 12; k++) {
      const int c = p + dz[k] * nx + dx[k];
      const double* a = T + (c < 0 ? 0 : c >= n ? n - 1 : c);
      t[k] = SC1 ? gld_sc1(a) : gld(a);
    }
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < 12; k++)
      if (z + dz[k] < nz && t[k] == t[k]) m |= 1u << k;
    vm = m;
    t0 = t[0]; t1 = t[1]; t2 = t[2]; t3 = t[3]; t4 = t[4]; t5 = t[5];
    t6 = t[6]; t7 = t[7]; t8 = t[8]; t9 = t[9]; t10 = t[10]; t11 = t[11];
  }
  AF_DEV void load(const double* T, int nz, int nx, int z, int x) { load_t<false>(T, nz, nx, z, x); }
  // the cell at offset (dz, dx) now holds the valid value v (no-op outside the 12 positions)
  AF_DEV void patch(int dz, int dx, double v) {
    const int ad = abs(dz) + abs(dx);
    if (ad == 0 || ad > 2 || (dz != 0 && dx != 0 && (abs(dz) != 1 || abs(dx) != 1))) return;
    const int k = NbField::slot(dz, dx);
    vm |= 1u << k;
    t0 = k == 0 ? v : t0; t1 = k == 1 ? v : t1; t2 = k == 2 ? v : t2; t3 = k == 3 ? v : t3;
    t4 = k == 4 ? v : t4; t5 = k == 5 ? v : t5; t6 = k == 6 ? v : t6; t7 = k == 7 ? v : t7;
    t8 = k == 8 ? v : t8; t9 = k == 9 ? v : t9; t10 = k == 10 ? v : t10; t11 = k == 11 ? v : t11;
  }
  // As load(), with sc1 loads (cells another workgroup of the launch writes)
  AF_DEV void load_sc1(const double* T, int nz, int nx, int z, int x) { load_t<true>(T, nz, nx, z, x); }
  // From a status-coded grid in LDS (the init kernel's stage grids / prefix window): validity =
  // inside rows [z0, z1] and columns [x0, x1] (else never-relaxed: nsts -1) and status >= 0;
  // the 24 LDS reads are issued together instead of as update()'s chain of dependent reads.
  AF_DEV void load_lds(const double* T, const short* S, int z0, int x0, int z1, int x1, int w, int z, int x) {
    iz = z;
    ix = x;
    const int dz[12] = {0, 0, 0, 0, -2, -1, 1, 2, -1, -1, 1, 1};
    const int dx[12] = {-2, -1, 1, 2, 0, 0, 0, 0, -1, 1, -1, 1};
    double t[12];
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < 12; k++) {
      const int zz = z + dz[k], xx = x + dx[k];
      const bool in = zz >= z0 && zz <= z1 && xx >= x0 && xx <= x1;
      const int c = in ? (zz - z0) * w + (xx - x0) : 0;
      t[k] = T[c];
      const int s = S[c];
      if (in && s >= 0) m |= 1u << k;
      if (!in) t[k] = 0.0;
    }
    vm = m;
    t0 = t[0]; t1 = t[1]; t2 = t[2]; t3 = t[3]; t4 = t[4]; t5 = t[5];
    t6 = t[6]; t7 = t[7]; t8 = t[8]; t9 = t[9]; t10 = t[10]; t11 = t[11];
  }
};

}  // namespace af
