// local_ops.h — the reference's local operators as templated device functions.
//
//   update()   — ALI locally-interpolated wavefront update, Anis_TTF_rays.py:904-1410
//   fouds18()  — multi-stencil quadratic fallback, Anis_TTF_rays.py:240-901
//
// F is a field accessor with  int st(long z, long x)  (node status; rows past the array read -1,
// the reference's padded stage-1 semantics) and  double tt(long z, long x).  Validity in update()
// is st >= 0 (alive or close), "known" in fouds18() is st == 0, exactly as in the reference.
// Material is read only at the target cell (CellMat), as in the reference.
#pragma once
#include <type_traits>
#include "device_common.h"

namespace af {

// fouds18_A()'s stencil-family slowness q (group velocity at 0, 45, -27, +27 deg off the cell's
// orientation, :281-300 and the three later families); a function of the cell's material only
AF_DEV double fouds18_slowness(const DevModel& M, const CellMat& cm, int q) {
    const double veln = cm.veln;
    double e = q == 0 ? pymod(0 - veln, 180)
             : q == 1 ? (double)pyround(pymod(45 - veln, 180))
             : q == 2 ? pymod(-27.0 - veln, 180) : pymod(27.0 - veln, 180);
    return 1.0 / group_vel_cell(M, cm, e);
}

// pre: the four slownesses of the cell's material precomputed by fouds18_slowness() (the band
// kernels read them from DevModel::mslo: the group-velocity code is the register-heaviest part of
// fouds18_A(), and the persistent kernels cannot afford its registers in the step loop), or null.
// PRE_ONLY: the caller guarantees pre != null, so the group-velocity code is not compiled in at all
// (fouds18_A() alone then needs 87 VGPRs instead of 181)
//
// fouds18_part(): the four stencil families' minima over the candidates of one PART (0..3: the
// family's candidate number part, -1: all of them; +inf where a family has no candidate), so that
// four lanes can evaluate one cell and combine their parts (fouds18_combine, the reference's
// combination :696-897).  Each family's result is a minimum over its candidates (the reference's
// running min, order-free: no candidate is NaN), so any split gives the same bits.
struct F18Part {
    double m[4];
};
template <bool PRE_ONLY = false, class F>
AF_DEV F18Part fouds18_part(const F& f, const DevModel& M, const CellMat& cm, long iz, long ix, double dnx,
                            double dnz, long nnx, long nnz, const double* pre, int part) {
    F18Part P;
#define N_(z, x) f.st((z), (x))
#define T_(z, x) f.tt((z), (x))
    /* ---- 0 deg stencil (:281-459) ---- */
    int tsw1 = 0;
    double travm = 0;
    /* the four stencil families' slownesses, computed unconditionally in the reference */
    double slo0 = 0, slo1 = 0, slo2 = 0, slo3 = 0;
    if (PRE_ONLY || pre) {
        slo0 = gld(pre);
        slo1 = gld(pre + 1);
        slo2 = gld(pre + 2);
        slo3 = gld(pre + 3);
    } else if constexpr (!PRE_ONLY) {
#pragma unroll 1
        for (int q = 0; q < 4; q++) {
            double g = fouds18_slowness(M, cm, q);
            if (q == 0) slo0 = g;
            else if (q == 1) slo1 = g;
            else if (q == 2) slo2 = g;
            else slo3 = g;
        }
    }
    double slown = slo0;
    #pragma unroll 1
    for (int jj_ = 0; jj_ < 2; jj_++) {
        long j = jj_ == 0 ? ix - 1 : ix + 1;
        if (0 <= j && j <= nnx - 1) {
            int swj = -1;
            long j2;
            if (j == ix - 1) {
                j2 = j - 1;
                if (j2 >= 0 && N_(iz, j2) == 0) swj = 0;
            } else {
                j2 = j + 1;
                if (j2 <= nnx - 1 && N_(iz, j2) == 0) swj = 0;
            }
            if (N_(iz, j) == 0 && swj == 0) {
                swj = -1;
                if (T_(iz, j) >= T_(iz, j2)) swj = 0;
            } else {
                swj = -1;
            }
            #pragma unroll 1
            for (int kk_ = 0; kk_ < 2; kk_++) {
                long k = kk_ == 0 ? iz - 1 : iz + 1;
                if (0 <= k && k <= nnz - 1 && (part < 0 || part == jj_ * 2 + kk_)) {
                    int swk = -1;
                    long k2;
                    if (k == iz - 1) {
                        k2 = k - 1;
                        if (k2 >= 0 && N_(k2, ix) == 0) swk = 0;
                    } else {
                        k2 = k + 1;
                        if (k2 <= nnz - 1 && N_(k2, ix) == 0) swk = 0;
                    }
                    if (N_(k, ix) == 0 && swk == 0) {
                        swk = -1;
                        if (T_(k, ix) >= T_(k2, ix)) swk = 0;
                    } else {
                        swk = -1;
                    }
                    int swsol = 0;
                    double a = 0, b = 0, c = 0, tref = 0, tdiv = 1, u, v;
                    (void)v;
                    if (swj == 0) {
                        swsol = 1;
                        if (swk == 0) {
                            u = 2.0 * dnx;
                            a = 18;
                            b = -6 * (4.0 * T_(iz, j) - T_(iz, j2) + 4.0 * T_(k, ix) - T_(k2, ix));
                            double p = 4.0 * T_(iz, j) - T_(iz, j2), q = 4.0 * T_(k, ix) - T_(k2, ix);
                            c = p * p + q * q - 4 * (u * u) * (slown * slown);
                            tref = 0.0; tdiv = 1.0;
                        } else if (N_(k, ix) == 0) {
                            u = dnz; v = 2.0 * dnx;
                            a = 18;
                            b = -6.0 * (3.0 * T_(k, ix) + 4.0 * T_(iz, j) - T_(iz, j2));
                            double p = 3.0 * T_(k, ix), q = 4.0 * T_(iz, j) - T_(iz, j2);
                            c = p * p + q * q - 4 * (v * v) * (slown * slown);
                            tref = 0.0; tdiv = 1.0;
                        } else {
                            u = 2.0 * dnx;
                            a = 1.0; b = 0.0;
                            c = -(u * u) * (slown * slown);
                            tref = 4.0 * T_(iz, j) - T_(iz, j2);
                            tdiv = 1.0; /* tdiv=3.0 is overwritten by tdiv=1.0 (:389,:395) */
                        }
                    } else if (N_(iz, j) == 0) {
                        swsol = 1;
                        if (swk == 0) {
                            u = dnx;
                            double em = 3.0 * T_(iz, j) + 4.0 * T_(k, ix) - T_(k2, ix);
                            a = 18; b = -6.0 * em;
                            double p = 3.0 * T_(iz, j), q = 4.0 * T_(k, ix) - T_(k2, ix);
                            c = p * p + q * q - 3 * 4 * (u * u) * (slown * slown);
                            tref = 0.0; tdiv = 1.0;
                        } else if (N_(k, ix) == 0) {
                            u = dnx; v = dnz;
                            a = 2;
                            b = -2 * (T_(k, ix) + T_(iz, j));
                            double w = u * slown;
                            c = T_(k, ix) * T_(k, ix) + T_(iz, j) * T_(iz, j) - w * w;
                            tref = 0.0; tdiv = 1.0;
                        } else {
                            a = 1.0; b = 0.0;
                            double w = T_(iz, j) + slown * dnx;
                            c = -(w * w);
                            tref = 0.0; tdiv = 1.0;
                        }
                    } else {
                        if (swk == 0) {
                            swsol = 1;
                            u = 2.0 * dnz;
                            a = 1.0; b = 0.0;
                            c = -(u * u) * (slown * slown);
                            tref = 4.0 * T_(k, ix) - T_(k2, ix);
                            tdiv = 3.0;
                        } else if (N_(k, ix) == 0) {
                            swsol = 1;
                            a = 1.0; b = 0.0;
                            double w = T_(k, ix) + slown * dnz;
                            c = -(w * w);
                            tref = 0.0; tdiv = 1.0;
                        }
                    }
                    if (swsol == 1) {
                        double rd1 = b * b - 4.0 * a * c;
                        if (rd1 < 0) rd1 = 0;
                        double tdsh = (-b + sqrt(rd1)) / (2.0 * a);
                        double trav = (tref + tdsh) / tdiv;
                        if (tsw1 == 1) travm = (travm < trav) ? travm : trav;
                        else { travm = trav; tsw1 = 1; }
                    }
                }
            }
        }
    }
    P.m[0] = tsw1 ? travm : INFINITY;
    /* ---- 45 deg stencil (:467-696) ---- */
    int tsw2 = 0;
    double travmd = 0;
    slown = slo1;
    double mf2 = sqrt(2.0);
    #pragma unroll 1
    for (int jj_ = 0; jj_ < 2; jj_++) {
        long j = (jj_ == 0) ? ix - 1 : ix + 1;
        long k = (j == ix - 1) ? iz + 1 : iz - 1;
        if (0 <= j && j <= nnx - 1 && 0 <= k && k <= nnz - 1) {
            int swdiag = -1;
            long j2 = 0, k2 = 0;
            if (j == ix - 1) {
                j2 = j - 1; k2 = k + 1;
                if (j2 >= 0 && k2 <= nnz - 1 && N_(k2, j2) == 0) swdiag = 0;
            } else {
                j2 = j + 1; k2 = k - 1;
                if (j2 <= nnx - 1 && k2 >= 0 && N_(k2, j2) == 0) swdiag = 0;
            }
            if (N_(k, j) == 0 && swdiag == 0) {
                swdiag = -1;
                if (T_(k, j) >= T_(k2, j2)) swdiag = 0;
            } else {
                swdiag = -1;
            }
            #pragma unroll 1
            for (int q_ = 0; q_ < 2; q_++) {
                long jj = (q_ == 0) ? ix - 1 : ix + 1;
                long kk = (jj == ix - 1) ? iz - 1 : iz + 1;
                if (0 <= jj && jj <= nnx - 1 && 0 <= kk && kk <= nnz - 1 && (part < 0 || part == jj_ * 2 + q_)) {
                    int swskew = -1;
                    long jj2, kk2;
                    if (jj == ix - 1) {
                        jj2 = jj - 1; kk2 = kk - 1;
                        if (jj2 >= 0 && kk2 >= 0 && N_(kk2, jj2) == 0) swskew = 0;
                    } else {
                        jj2 = jj + 1; kk2 = kk + 1;
                        if (jj2 <= nnx - 1 && kk2 <= nnz - 1 && N_(kk2, jj2) == 0) swskew = 0;
                    }
                    if (N_(kk, jj) == 0 && swskew == 0) {
                        swskew = -1;
                        if (T_(kk, jj) >= T_(kk2, jj2)) swskew = 0;
                    } else {
                        swskew = -1;
                    }
                    int swsol = 0;
                    double a = 0, b = 0, c = 0, tref = 0, tdiv = 1, u, v;
                    (void)v;
                    if (swdiag == 0) {
                        swsol = 1;
                        if (swskew == 0) {
                            u = 2.0 * mf2 * dnx;
                            a = 18.0;
                            b = -6.0 * (4.0 * T_(k, j) - T_(k2, j2) + 4.0 * T_(kk, jj) - T_(kk2, jj2));
                            double p = 4.0 * T_(k, j) - T_(k2, j2), q = 4.0 * T_(kk, jj) - T_(kk2, jj2);
                            c = p * p + q * q - 4 * (u * u) * (slown * slown);
                            tref = 0; tdiv = 1.0;
                        } else if (N_(kk, jj) == 0) {
                            u = mf2 * dnz; v = 2.0 * mf2 * dnx;
                            a = 18;
                            b = -6.0 * (3.0 * T_(kk, jj) + 4.0 * T_(k, j) - T_(k2, j2));
                            double p = 3.0 * T_(kk, jj), q = 4.0 * T_(k, j) - T_(k2, j2);
                            c = p * p + q * q - 4 * (v * v) * (slown * slown);
                            tref = 0.0; tdiv = 1.0;
                        } else {
                            u = mf2 * 2.0 * dnx;
                            a = 1.0; b = 0.0;
                            double w = u * slown;
                            c = -1.0 * (w * w);
                            tref = 4.0 * T_(k, j) - T_(k2, j2);
                            tdiv = 3.0;
                        }
                    } else if (N_(k, j) == 0) {
                        swsol = 1;
                        if (swskew == 0) {
                            u = mf2 * dnx; v = mf2 * 2.0 * dnz;
                            double em = 3.0 * T_(k, j) + 4.0 * T_(kk, jj) - T_(kk2, jj2);
                            a = 18; b = -6.0 * em;
                            double p = 3.0 * T_(k, j), q = 4.0 * T_(kk, jj) - T_(kk2, jj2);
                            c = p * p + q * q - 3 * 4 * (u * u) * (slown * slown);
                            tref = 0.0; tdiv = 1.0;
                        } else if (N_(kk, jj) == 0) {
                            u = mf2 * dnx; v = mf2 * dnz;
                            a = 2;
                            b = -2 * (T_(kk, jj) + T_(k, j));
                            double w = u * slown;
                            c = T_(kk, jj) * T_(kk, jj) + T_(k, j) * T_(k, j) - 4.0 / 9.0 * (w * w);
                            tref = 0.0; tdiv = 1.0;
                        } else {
                            u = mf2 * dnx;
                            a = 1.0; b = 0.0;
                            double w = T_(k, j) + slown * u;
                            c = -(w * w);
                            tref = 0; tdiv = 1.0;
                        }
                    } else {
                        if (swskew == 0) {
                            swsol = 1;
                            u = 2.0 * mf2 * dnz;
                            a = 1.0; b = 0.0;
                            c = -(u * u) * (slown * slown);
                            tref = 4.0 * T_(kk, jj) - T_(kk2, jj2);
                            tdiv = 3.0;
                        } else if (N_(kk, jj) == 0) {
                            swsol = 1;
                            u = mf2 * dnx;
                            a = 1.0; b = 0.0;
                            c = -(slown * slown) * (u * u);
                            tref = T_(kk, jj);
                            tdiv = 1.0;
                        }
                    }
                    if (swsol == 1) {
                        double rd1 = b * b - 4.0 * a * c;
                        if (rd1 > 0) {
                            double tdsh = (-b + sqrt(rd1)) / (2.0 * a);
                            double trav = (tref + tdsh) / tdiv;
                            if (tsw2 == 1) travmd = (travmd < trav) ? travmd : trav;
                            else { travmd = trav; tsw2 = 1; }
                        }
                    }
                }
            }
        }
    }
    P.m[1] = tsw2 ? travmd : INFINITY;

    /* ---- atan(1/2) stencils (:698-897) ---- */
    #pragma unroll 1
    for (int pass = 0; pass < 2; pass++) {
        slown = pass == 0 ? slo2 : slo3;
        double m5 = sqrt(5.0);
        /* j_vec/k_vec of :740-741 (pass 0) and :839-840 (pass 1) as offsets (no indexed arrays) */
#define JV(l) (ix + (pass == 0 ? ((l) % 4 == 0 ? -1 : (l) == 1 ? 2 : (l) == 2 ? 1 : -2) \
                               : ((l) % 4 == 0 ? 1 : (l) == 1 ? 2 : (l) == 2 ? -1 : -2)))
#define KV(l) (iz + (pass == 0 ? ((l) % 4 == 0 ? -2 : (l) == 1 ? -1 : (l) == 2 ? 2 : 1) \
                               : ((l) % 4 == 0 ? -2 : (l) == 1 ? 1 : (l) == 2 ? 2 : -1)))
        int tsw = 0;
        double tm = 0;
        #pragma unroll 1
        for (int lp = 0; lp < 4; lp++) {
            long j = JV(lp), k = KV(lp), jj = JV(lp + 1), kk = KV(lp + 1);
            if (0 <= j && j <= nnx - 1 && 0 <= k && k <= nnz - 1 && 0 <= jj && jj <= nnx - 1 && 0 <= kk &&
                kk <= nnz - 1 && (part < 0 || part == lp)) {
                int swsol = 0;
                double a = 0, b = 0, c = 0, tref = 0, u;
                if (N_(k, j) == 0) {
                    swsol = 1;
                    if (N_(kk, jj) == 0) {
                        u = m5 * dnx;
                        a = 2;
                        b = -2 * (T_(kk, jj) + T_(k, j));
                        double w = u * slown;
                        c = T_(kk, jj) * T_(kk, jj) + T_(k, j) * T_(k, j) - 2 * (w * w);
                        tref = 0.0;
                    } else {
                        u = m5 * dnx;
                        a = 1; b = 0;
                        double w = slown * u;
                        c = -(w * w);
                        tref = T_(k, j);
                    }
                } else if (N_(kk, jj) == 0) {
                    swsol = 1;
                    u = m5 * dnx;
                    a = 1; b = 0;
                    double w = slown * u;
                    c = -(w * w);
                    tref = T_(kk, jj);
                }
                if (swsol == 1) {
                    double rd1 = b * b - 4 * a * c;
                    if (rd1 < 0) rd1 = 0;
                    double tdsh = (-b + sqrt(rd1)) / (2.0 * a);
                    double trav = tref + tdsh;
                    if (tsw == 1) tm = (trav < tm) ? trav : tm;
                    else { tm = trav; tsw = 1; }
                }
            }
        }
        P.m[2 + pass] = tsw ? tm : INFINITY;
    }
#undef JV
#undef KV
    return P;
#undef N_
#undef T_
}

// the minimum of two parts' family results (lanes of one cell)
AF_DEV F18Part f18_min(const F18Part& a, const F18Part& b) {
    F18Part r;
    for (int k = 0; k < 4; k++) r.m[k] = (a.m[k] < b.m[k]) ? a.m[k] : b.m[k];
    return r;
}

// the reference's combination of the families (:696-697, :798-800, :895-897) and of the current ttn
AF_DEV double fouds18_combine(const F18Part& P, double cur) {
    const double travm = P.m[0] == INFINITY ? 0.0 : P.m[0];
    double travmd = P.m[1] == INFINITY ? 0.0 : P.m[1];
    if (travmd != 0) travmd = (travm < travmd) ? travm : travmd;
    else travmd = travm;
    double travmt = P.m[2] == INFINITY ? 0.0 : P.m[2];
    if (travmt != 0) travmt = (travmt < travmd) ? travmt : travmd;
    else travmt = travmd;
    double travms = P.m[3] == INFINITY ? 0.0 : P.m[3];
    if (travms != 0) travms = (travmt < travms) ? travmt : travms;
    else travms = travmt;
    if (cur != 0) travms = (travms < cur) ? travms : cur;
    return travms;
}

template <bool PRE_ONLY = false, class F>
AF_DEV double fouds18(const F& f, const DevModel& M, const CellMat& cm, long iz, long ix, double dnx, double dnz,
                      long nnx, long nnz, const double* pre = nullptr) {
    return fouds18_combine(fouds18_part<PRE_ONLY>(f, M, cm, iz, ix, dnx, dnz, nnx, nnz, pre, -1), f.tt(iz, ix));
}


// update() index type: grid coordinates fit in int; the long of the reference's numba code
// only widens the integer arithmetic (the doubles formed from the coordinates are the same)
#ifndef AF_UPD_IDX
#define AF_UPD_IDX int
#endif
// update()'s triangular-stencil stage (:1146-1366) and its inputs/outputs, shared by the
// reference-form square stage (update_ref) and the branch-free one for register neighbourhoods
// (update_nb).  W holds the parameters of the one wavefront_angle_dist() call.
template <class I>
struct UpdW {
    I x1, x2, x3, z1, z2, z3;
    double y1, y2, y3;
    bool have;
};
template <class F, class I>
AF_DEV void upd_tri(const F& f, I iz, I ix, I nnz, I nnx, int& sno, double& min_diff, double& diff, UpdW<I>& w,
                    double& wt, double& angle, double& dist) {
#define N_(z, x) f.st((z), (x))
#define T_(z, x) f.tt((z), (x))
#define SETW(a1, a2, a3, b1, b2, b3, c1, c2, c3) \
    do { w.x1 = (a1); w.x2 = (a2); w.x3 = (a3); w.z1 = (b1); w.z2 = (b2); w.z3 = (b3); \
         w.y1 = (c1); w.y2 = (c2); w.y3 = (c3); w.have = true; } while (0)
    bool& have_w = w.have;
        /* triangular stencils :1146-1366 */
        int tp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (ix > 1) { if (N_(iz, ix - 2) >= 0) { tp[4]++; tp[7]++; } }
        if (ix > 0) {
            if (N_(iz, ix - 1) >= 0) { tp[4]++; tp[7]++; }
            if (iz > 0) { if (N_(iz - 1, ix - 1) >= 0) { tp[2]++; tp[7]++; } }
            if (iz < nnz - 1) { if (N_(iz + 1, ix - 1) >= 0) { tp[3]++; tp[4]++; } }
        }
        if (ix < nnx - 2) { if (N_(iz, ix + 2) >= 0) { tp[5]++; tp[6]++; } }
        if (ix < nnx - 1) {
            if (N_(iz, ix + 1) >= 0) { tp[5]++; tp[6]++; }
            if (iz > 0) { if (N_(iz - 1, ix + 1) >= 0) { tp[1]++; tp[6]++; } }
            if (iz < nnz - 1) { if (N_(iz + 1, ix + 1) >= 0) { tp[0]++; tp[5]++; } }
        }
        if (iz > 1) { if (N_(iz - 2, ix) >= 0) { tp[1]++; tp[2]++; } }
        if (iz > 0) { if (N_(iz - 1, ix) >= 0) { tp[1]++; tp[2]++; } }
        if (iz < nnz - 2) { if (N_(iz + 2, ix) >= 0) { tp[0]++; tp[3]++; } }
        if (iz < nnz - 1) { if (N_(iz + 1, ix) >= 0) { tp[0]++; tp[3]++; } }

        if (sno == -1) min_diff = 1000000.0;
        sno = -2;
        const double s2m1 = sqrt(2.0) - 1, tms2 = 2 - sqrt(2.0);
#define TRI(id, ca, cb, cc)                                                                   \
    if (tp[id] == 3) {                                                                        \
        double A_ = (ca), B_ = (cb), C_ = (cc);                                               \
        if (A_ < ((B_ < C_) ? B_ : C_)) {                                                     \
            diff = fabs(s2m1 * A_ + tms2 * B_ - C_);                                          \
            if (diff < min_diff) { sno = id; min_diff = diff; }                               \
        }                                                                                     \
    }
        TRI(0, T_(iz + 2, ix), T_(iz + 1, ix), T_(iz + 1, ix + 1))
        TRI(1, T_(iz - 2, ix), T_(iz - 1, ix), T_(iz - 1, ix + 1))
        TRI(2, T_(iz - 2, ix), T_(iz - 1, ix), T_(iz - 1, ix - 1))
        TRI(3, T_(iz + 2, ix), T_(iz + 1, ix), T_(iz + 1, ix - 1))
        TRI(4, T_(iz, ix - 2), T_(iz, ix - 1), T_(iz + 1, ix - 1))
        TRI(5, T_(iz, ix + 2), T_(iz, ix + 1), T_(iz + 1, ix + 1))
        TRI(6, T_(iz, ix + 2), T_(iz, ix + 1), T_(iz - 1, ix + 1))
        TRI(7, T_(iz, ix - 2), T_(iz, ix - 1), T_(iz - 1, ix - 1))
#undef TRI
        /* NOTE: the reference's min(b, c) for the guard: numba min(b,c) -> b if not (c < b) */
        if (sno != -2) {
            switch (sno) {
            case 0:
                if (T_(iz + 1, ix) < T_(iz + 1, ix + 1)) {
                    if (ix == 0) { angle = 90.; dist = 1.; have_w = false; }
                    else SETW(ix, ix, ix + 1, iz + 2, iz + 1, iz + 1, T_(iz + 2, ix), T_(iz + 1, ix), T_(iz + 1, ix + 1));
                } else {
                    SETW(ix, ix + 1, ix, iz + 2, iz + 1, iz + 1, T_(iz + 2, ix), T_(iz + 1, ix + 1), T_(iz + 1, ix));
                }
                wt = T_(iz + 1, ix + 1); /* SURVEY B-D15 */
                break;
            case 1:
                if (T_(iz - 1, ix) < T_(iz - 1, ix + 1)) {
                    if (ix == 0) { angle = 90.; dist = 1.; have_w = false; }
                    else SETW(ix, ix, ix + 1, iz - 2, iz - 1, iz - 1, T_(iz - 2, ix), T_(iz - 1, ix), T_(iz - 1, ix + 1));
                    wt = T_(iz - 1, ix);
                } else {
                    SETW(ix, ix + 1, ix, iz - 2, iz - 1, iz - 1, T_(iz - 2, ix), T_(iz - 1, ix + 1), T_(iz - 1, ix));
                    wt = T_(iz - 1, ix + 1);
                }
                break;
            case 2:
                if (T_(iz - 1, ix) < T_(iz - 1, ix - 1)) {
                    if (ix == nnx - 1) { angle = 90.; dist = 1.; have_w = false; }
                    else SETW(ix, ix, ix - 1, iz - 2, iz - 1, iz - 1, T_(iz - 2, ix), T_(iz - 1, ix), T_(iz - 1, ix - 1));
                    wt = T_(iz - 1, ix);
                } else {
                    SETW(ix, ix - 1, ix, iz - 2, iz - 1, iz - 1, T_(iz - 2, ix), T_(iz - 1, ix - 1), T_(iz - 1, ix));
                    wt = T_(iz - 1, ix - 1);
                }
                break;
            case 3:
                if (T_(iz + 1, ix) < T_(iz + 1, ix - 1)) {
                    if (ix == nnx - 1) { angle = 90.; dist = 1.; have_w = false; }
                    else SETW(ix, ix, ix - 1, iz + 2, iz + 1, iz + 1, T_(iz + 2, ix), T_(iz + 1, ix), T_(iz + 1, ix - 1));
                    wt = T_(iz + 1, ix);
                } else {
                    SETW(ix, ix - 1, ix, iz + 2, iz + 1, iz + 1, T_(iz + 2, ix), T_(iz + 1, ix - 1), T_(iz + 1, ix));
                    wt = T_(iz + 1, ix - 1);
                }
                break;
            case 4:
                if (T_(iz, ix - 1) < T_(iz + 1, ix - 1)) {
                    if (iz == 0) { angle = 0.; dist = 1.; have_w = false; }
                    else SETW(ix - 2, ix - 1, ix - 1, iz, iz, iz + 1, T_(iz, ix - 2), T_(iz, ix - 1), T_(iz + 1, ix - 1));
                    wt = T_(iz, ix - 1);
                } else {
                    SETW(ix - 2, ix - 1, ix - 1, iz, iz + 1, iz, T_(iz, ix - 2), T_(iz + 1, ix - 1), T_(iz, ix - 1));
                    wt = T_(iz + 1, ix - 1);
                }
                break;
            case 5:
                if (T_(iz, ix + 1) < T_(iz + 1, ix + 1)) {
                    if (iz == 0) { angle = 0.; dist = 1.; have_w = false; }
                    else SETW(ix + 2, ix + 1, ix + 1, iz, iz, iz + 1, T_(iz, ix + 2), T_(iz, ix + 1), T_(iz + 1, ix + 1));
                    wt = T_(iz, ix + 1);
                } else {
                    SETW(ix + 2, ix + 1, ix + 1, iz, iz + 1, iz, T_(iz, ix + 2), T_(iz + 1, ix + 1), T_(iz, ix + 1));
                    wt = T_(iz + 1, ix + 1);
                }
                break;
            case 6:
                if (T_(iz, ix + 1) < T_(iz - 1, ix + 1)) {
                    if (iz == nnz - 1) { angle = 0.; dist = 1.; have_w = false; }
                    else SETW(ix + 2, ix + 1, ix + 1, iz, iz, iz - 1, T_(iz, ix + 2), T_(iz, ix + 1), T_(iz - 1, ix + 1));
                    wt = T_(iz, ix + 1);
                } else {
                    SETW(ix + 2, ix + 1, ix + 1, iz, iz - 1, iz, T_(iz, ix + 2), T_(iz - 1, ix + 1), T_(iz, ix + 1));
                    wt = T_(iz - 1, ix + 1);
                }
                break;
            case 7:
                if (T_(iz, ix - 1) < T_(iz - 1, ix - 1)) {
                    if (iz == nnz - 1) { angle = 0.; dist = 1.; have_w = false; }
                    else SETW(ix - 2, ix - 1, ix - 1, iz, iz, iz - 1, T_(iz, ix - 2), T_(iz, ix - 1), T_(iz - 1, ix - 1));
                    wt = T_(iz, ix - 1);
                } else {
                    SETW(ix - 2, ix - 1, ix - 1, iz, iz - 1, iz, T_(iz, ix - 2), T_(iz - 1, ix - 1), T_(iz, ix - 1));
                    wt = T_(iz - 1, ix - 1);
                }
                break;
            }
            sno += 8;
        }
#undef SETW
#undef N_
#undef T_
}

// the phase velocity of the chosen stencil's wavefront direction and the result (:1368-1410)
template <class I>
AF_DEV double upd_finish(const DevModel& M, const CellMat& cm, I ix, I iz, const UpdW<I>& w, double wt,
                         double angle, double dist, double dnx) {
    if (w.have) wad(ix, iz, w.x1, w.x2, w.x3, w.z1, w.z2, w.z3, w.y1, w.y2, w.y3, angle, dist);
    if (dist != -1.0) {
        double effa = pymod(cm.veln - angle, 180);
        double velocity;
        if (cm.velpn != 0 || cm.stif == nullptr) velocity = table_vel(M.ptab, M.ncol, effa, cm.velpn, cm.vm);
        else velocity = christoffel_phase(cm.stif, effa, cm.vm);
        return wt + (dist * dnx / velocity);
    }
    return -1.0;
}

template <class F>
AF_DEV double update_ref(const F& f, const DevModel& M, const CellMat& cm, AF_UPD_IDX iz, AF_UPD_IDX ix, double dnx,
                     AF_UPD_IDX nnz, AF_UPD_IDX nnx) {
#define N_(z, x) f.st((z), (x))
#define T_(z, x) f.tt((z), (x))
    int sp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (ix > 1) { if (N_(iz, ix - 2) >= 0) sp[3]++; }
    if (ix > 0) {
        if (N_(iz, ix - 1) >= 0) { sp[4]++; sp[7]++; }
        if (iz > 0) { if (N_(iz - 1, ix - 1) >= 0) { sp[0]++; sp[3]++; sp[4]++; } }
        if (iz < nnz - 1) { if (N_(iz + 1, ix - 1) >= 0) { sp[2]++; sp[3]++; sp[7]++; } }
    }
    if (ix < nnx - 2) { if (N_(iz, ix + 2) >= 0) sp[1]++; }
    if (ix < nnx - 1) {
        if (N_(iz, ix + 1) >= 0) { sp[5]++; sp[6]++; }
        if (iz > 0) { if (N_(iz - 1, ix + 1) >= 0) { sp[0]++; sp[1]++; sp[5]++; } }
        if (iz < nnz - 1) { if (N_(iz + 1, ix + 1) >= 0) { sp[1]++; sp[2]++; sp[6]++; } }
    }
    if (iz > 1) { if (N_(iz - 2, ix) >= 0) sp[0]++; }
    if (iz > 0) { if (N_(iz - 1, ix) >= 0) { sp[4]++; sp[5]++; } }
    if (iz < nnz - 2) { if (N_(iz + 2, ix) >= 0) sp[2]++; }
    if (iz < nnz - 1) { if (N_(iz + 1, ix) >= 0) { sp[6]++; sp[7]++; } }

    int sno = -1;
    double min_diff = 1000000.0, diff;
    if (sp[0] == 3) { diff = fabs(T_(iz - 1, ix - 1) - T_(iz - 1, ix + 1)); if (diff < min_diff) { sno = 0; min_diff = diff; } }
    if (sp[1] == 3) { diff = fabs(T_(iz - 1, ix + 1) - T_(iz + 1, ix + 1)); if (diff < min_diff) { sno = 1; min_diff = diff; } }
    if (sp[2] == 3) { diff = fabs(T_(iz + 1, ix - 1) - T_(iz + 1, ix + 1)); if (diff < min_diff) { sno = 2; min_diff = diff; } }
    if (sp[3] == 3) { diff = fabs(T_(iz - 1, ix - 1) - T_(iz + 1, ix - 1)); if (diff < min_diff) { sno = 3; min_diff = diff; } }
    if (sp[4] == 3) { diff = fabs(T_(iz, ix - 1) - T_(iz - 1, ix)); if (diff < min_diff) { sno = 4; min_diff = diff; } }
    if (sp[5] == 3) { diff = fabs(T_(iz - 1, ix) - T_(iz, ix + 1)); if (diff < min_diff) { sno = 5; min_diff = diff; } }
    if (sp[6] == 3) { diff = fabs(T_(iz + 1, ix) - T_(iz, ix + 1)); if (diff < min_diff) { sno = 6; min_diff = diff; } }
    if (sp[7] == 3) { diff = fabs(T_(iz, ix - 1) - T_(iz + 1, ix)); if (diff < min_diff) { sno = 7; min_diff = diff; } }

    double angle = 0.0, dist = -1.0, wt = 0.0;
    /* wavefront_angle_dist is evaluated once, after stencil selection, on the parameters of the
       stencil that the reference's last wavefront_angle_dist call would use (same result, one
       inlined instance instead of 32: keeps the kernels free of register spills) */
    bool have_w = false;
    AF_UPD_IDX wx1 = 0, wx2 = 0, wx3 = 0, wz1 = 0, wz2 = 0, wz3 = 0;
    double wy1 = 0, wy2 = 0, wy3 = 0;
#define SETW(a1, a2, a3, b1, b2, b3, c1, c2, c3) \
    do { wx1 = (a1); wx2 = (a2); wx3 = (a3); wz1 = (b1); wz2 = (b2); wz3 = (b3); \
         wy1 = (c1); wy2 = (c2); wy3 = (c3); have_w = true; } while (0)
    if (sno != -1) {
        /* square stencils :1039-1143 (both nsts sub-branches of stencils 0-3 are identical) */
        switch (sno) {
        case 0:
            if (T_(iz - 1, ix - 1) < T_(iz - 1, ix + 1)) {
                SETW(ix, ix - 1, ix + 1, iz - 2, iz - 1, iz - 1, T_(iz - 2, ix), T_(iz - 1, ix - 1), T_(iz - 1, ix + 1));
                wt = T_(iz - 1, ix - 1);
            } else {
                SETW(ix, ix + 1, ix - 1, iz - 2, iz - 1, iz - 1, T_(iz - 2, ix), T_(iz - 1, ix + 1), T_(iz - 1, ix - 1));
                wt = T_(iz - 1, ix + 1);
            }
            break;
        case 1:
            if (T_(iz - 1, ix + 1) < T_(iz + 1, ix + 1)) {
                SETW(ix + 2, ix + 1, ix + 1, iz, iz - 1, iz + 1, T_(iz, ix + 2), T_(iz - 1, ix + 1), T_(iz + 1, ix + 1));
                wt = T_(iz - 1, ix + 1);
            } else {
                SETW(ix + 2, ix + 1, ix + 1, iz, iz + 1, iz - 1, T_(iz, ix + 2), T_(iz + 1, ix + 1), T_(iz - 1, ix + 1));
                wt = T_(iz + 1, ix + 1);
            }
            break;
        case 2:
            if (T_(iz + 1, ix - 1) < T_(iz + 1, ix + 1)) {
                SETW(ix, ix - 1, ix + 1, iz + 2, iz + 1, iz + 1, T_(iz + 2, ix), T_(iz + 1, ix - 1), T_(iz + 1, ix + 1));
                wt = T_(iz + 1, ix - 1);
            } else {
                SETW(ix, ix + 1, ix - 1, iz + 2, iz + 1, iz + 1, T_(iz + 2, ix), T_(iz + 1, ix + 1), T_(iz + 1, ix - 1));
                wt = T_(iz + 1, ix + 1);
            }
            break;
        case 3:
            if (T_(iz - 1, ix - 1) < T_(iz + 1, ix - 1)) {
                SETW(ix - 2, ix - 1, ix - 1, iz, iz - 1, iz + 1, T_(iz, ix - 2), T_(iz - 1, ix - 1), T_(iz + 1, ix - 1));
                wt = T_(iz - 1, ix - 1);
            } else {
                SETW(ix - 2, ix - 1, ix - 1, iz, iz + 1, iz - 1, T_(iz, ix - 2), T_(iz + 1, ix - 1), T_(iz - 1, ix - 1));
                wt = T_(iz + 1, ix - 1);
            }
            break;
        case 4:
            if (T_(iz, ix - 1) < T_(iz - 1, ix)) {
                SETW(ix - 1, ix - 1, ix, iz - 1, iz, iz - 1, T_(iz - 1, ix - 1), T_(iz, ix - 1), T_(iz - 1, ix));
                wt = T_(iz, ix - 1);
            } else {
                SETW(ix - 1, ix, ix - 1, iz - 1, iz - 1, iz, T_(iz - 1, ix - 1), T_(iz - 1, ix), T_(iz, ix - 1));
                wt = T_(iz - 1, ix);
            }
            break;
        case 5:
            if (T_(iz - 1, ix) < T_(iz, ix + 1)) {
                SETW(ix + 1, ix, ix + 1, iz - 1, iz - 1, iz, T_(iz - 1, ix + 1), T_(iz - 1, ix), T_(iz, ix + 1));
                wt = T_(iz - 1, ix);
            } else {
                SETW(ix + 1, ix + 1, ix, iz - 1, iz, iz - 1, T_(iz - 1, ix + 1), T_(iz, ix + 1), T_(iz - 1, ix));
                wt = T_(iz, ix + 1);
            }
            break;
        case 6:
            if (T_(iz + 1, ix) < T_(iz, ix + 1)) {
                SETW(ix + 1, ix, ix + 1, iz + 1, iz + 1, iz, T_(iz + 1, ix + 1), T_(iz + 1, ix), T_(iz, ix + 1));
                wt = T_(iz + 1, ix);
            } else {
                SETW(ix + 1, ix + 1, ix, iz + 1, iz, iz + 1, T_(iz + 1, ix + 1), T_(iz, ix + 1), T_(iz + 1, ix));
                wt = T_(iz, ix + 1);
            }
            break;
        case 7:
            if (T_(iz, ix - 1) < T_(iz + 1, ix)) {
                SETW(ix - 1, ix - 1, ix, iz + 1, iz, iz + 1, T_(iz + 1, ix - 1), T_(iz, ix - 1), T_(iz + 1, ix));
                wt = T_(iz, ix - 1);
            } else {
                SETW(ix - 1, ix, ix - 1, iz + 1, iz + 1, iz, T_(iz + 1, ix - 1), T_(iz + 1, ix), T_(iz, ix - 1));
                wt = T_(iz + 1, ix);
            }
            break;
        }
    }

    if (sno == -1 || ix == 0 || ix == nnx - 1 || iz == 0 || iz == nnz - 1) {
        UpdW<AF_UPD_IDX> w{wx1, wx2, wx3, wz1, wz2, wz3, wy1, wy2, wy3, have_w};
        upd_tri(f, iz, ix, nnz, nnx, sno, min_diff, diff, w, wt, angle, dist);
#undef SETW
        return upd_finish(M, cm, ix, iz, w, wt, angle, dist, dnx);
    }
    UpdW<AF_UPD_IDX> w{wx1, wx2, wx3, wz1, wz2, wz3, wy1, wy2, wy3, have_w};
    return upd_finish(M, cm, ix, iz, w, wt, angle, dist, dnx);
#undef N_
#undef T_
}



// update() on a register neighbourhood (NbField / NbFieldT: t0..t11 and the validity mask vm,
// slots as NbField::slot): the same square-stencil stage as update_ref without branches — the
// sp[k] == 3 tests become mask tests (the bounds checks folded into the mask), the first-minimum
// selection keeps the reference's order and strict '<', and the chosen stencil's wavefront
// parameters are carried through the selection instead of a 16-way switch, so a wavefront does
// not serialise over its lanes' stencil cases.  The triangular stage and the velocity are shared
// with update_ref.  Bit-identical to update_ref (tools/micro/update_bench checksums, GPU tests).
// update()'s result is upd_finish() of the stencil stage's outputs: two calls whose stencil
// stages are equal give the same value (the init kernels' parallel relaxation relies on it)
struct UpdSel {
    UpdW<AF_UPD_IDX> w;
    double wt, angle, dist;
    AF_DEV bool same(const UpdSel& o) const {
        return w.have == o.w.have && w.x1 == o.w.x1 && w.x2 == o.w.x2 && w.x3 == o.w.x3 && w.z1 == o.w.z1 &&
               w.z2 == o.w.z2 && w.z3 == o.w.z3 && __double_as_longlong(w.y1) == __double_as_longlong(o.w.y1) &&
               __double_as_longlong(w.y2) == __double_as_longlong(o.w.y2) &&
               __double_as_longlong(w.y3) == __double_as_longlong(o.w.y3) &&
               __double_as_longlong(wt) == __double_as_longlong(o.wt) &&
               __double_as_longlong(angle) == __double_as_longlong(o.angle) &&
               __double_as_longlong(dist) == __double_as_longlong(o.dist);
    }
};

template <class F>
AF_DEV UpdSel update_nb_select(const F& f, AF_UPD_IDX iz, AF_UPD_IDX ix, AF_UPD_IDX nnz, AF_UPD_IDX nnx) {
    using I = AF_UPD_IDX;
    const bool l1 = ix > 0, l2 = ix > 1, r1 = ix < nnx - 1, r2 = ix < nnx - 2;
    const bool u1 = iz > 0, u2 = iz > 1, d1 = iz < nnz - 1, d2 = iz < nnz - 2;
    const unsigned inb = (l2 ? 1u : 0u) | (l1 ? 2u : 0u) | (r1 ? 4u : 0u) | (r2 ? 8u : 0u) | (u2 ? 16u : 0u) |
                         (u1 ? 32u : 0u) | (d1 ? 64u : 0u) | (d2 ? 128u : 0u) | (l1 && u1 ? 256u : 0u) |
                         (r1 && u1 ? 512u : 0u) | (l1 && d1 ? 1024u : 0u) | (r1 && d1 ? 2048u : 0u);
    const unsigned em = f.vm & inb;
    const double t[12] = {f.t0, f.t1, f.t2, f.t3, f.t4, f.t5, f.t6, f.t7, f.t8, f.t9, f.t10, f.t11};
    // square stencil k: apex, a, b slots; diff = |T_a - T_b|; the wavefront points are (apex, a, b)
    // when T_a < T_b, else (apex, b, a) (:1039-1143)
    constexpr int AP[8] = {4, 3, 7, 0, 8, 9, 11, 10};
    constexpr int SA[8] = {8, 9, 10, 8, 1, 5, 6, 1};
    constexpr int SB[8] = {9, 11, 11, 10, 5, 2, 2, 6};
    // slot -> (dz + 2) * 8 + (dx + 2)
    constexpr int OFF[12] = {16, 17, 19, 20, 2, 10, 26, 34, 9, 11, 25, 27};
    int sno = -1, code = 0;
    double min_diff = 1000000.0, diff = 0.0, yap = 0.0, ya = 0.0, yb = 0.0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const unsigned msk = (1u << AP[k]) | (1u << SA[k]) | (1u << SB[k]);
        const double d = fabs(t[SA[k]] - t[SB[k]]);
        if ((em & msk) == msk && d < min_diff) {
            sno = k;
            min_diff = d;
            yap = t[AP[k]];
            ya = t[SA[k]];
            yb = t[SB[k]];
            code = OFF[AP[k]] | (OFF[SA[k]] << 6) | (OFF[SB[k]] << 12);
        }
    }
    UpdSel r{UpdW<I>{0, 0, 0, 0, 0, 0, 0.0, 0.0, 0.0, false}, 0.0, 0.0, -1.0};
    if (sno >= 0) {
        const bool lo = ya < yb;
        const int pa = (code >> 6) & 63, pb = (code >> 12) & 63;
        const int p1 = code & 63, p2 = lo ? pa : pb, p3 = lo ? pb : pa;
        r.w.x1 = ix + (p1 & 7) - 2;
        r.w.z1 = iz + (p1 >> 3) - 2;
        r.w.x2 = ix + (p2 & 7) - 2;
        r.w.z2 = iz + (p2 >> 3) - 2;
        r.w.x3 = ix + (p3 & 7) - 2;
        r.w.z3 = iz + (p3 >> 3) - 2;
        r.w.y1 = yap;
        r.w.y2 = lo ? ya : yb;
        r.w.y3 = lo ? yb : ya;
        r.w.have = true;
        r.wt = r.w.y2;
    }
    if (sno == -1 || ix == 0 || ix == nnx - 1 || iz == 0 || iz == nnz - 1)
        upd_tri(f, iz, ix, nnz, nnx, sno, min_diff, diff, r.w, r.wt, r.angle, r.dist);
    return r;
}

// eight 4-bit fields, the first lowest
constexpr unsigned nib8(unsigned a, unsigned b, unsigned c, unsigned d, unsigned e, unsigned f, unsigned g,
                        unsigned h) {
    return a | b << 4 | c << 8 | d << 12 | e << 16 | f << 20 | g << 24 | h << 28;
}
static_assert(nib8(4, 3, 7, 0, 8, 9, 11, 10) == 0xab980734u, "nibble packing");
// twelve 4-bit fields, the first lowest
constexpr unsigned long long nib12(unsigned a, unsigned b, unsigned c, unsigned d, unsigned e, unsigned f,
                                   unsigned g, unsigned h, unsigned i, unsigned j, unsigned k, unsigned l) {
    return (unsigned long long)nib8(a, b, c, d, e, f, g, h) | (unsigned long long)(i | j << 4 | k << 8 | l << 12) << 32;
}

// DPP moves (gfx9 controls: quad_perm 0x00-0xff, row_mirror 0x140, row_half_mirror 0x141)
template <int CTRL>
AF_DEV int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
AF_DEV double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)dpp_i<CTRL>((int)b), hi = (unsigned)dpp_i<CTRL>((int)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
#ifndef AF_SEL_DPP
#define AF_SEL_DPP 1
#endif

// value of lane l (l wave-uniform)
AF_DEV double lane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)b, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// update_nb_select() spread over a wavefront (every lane calls it, wave-uniform arguments): lane
// k < 12 holds NbField slot k's value tk and validity vk; lane k < 8 forms square stencil k's
// |T_a - T_b| and a three-round min-reduction that keeps the lowest index on ties picks the
// stencil, which is the reference's first-minimum scan with strict '<' (:994-1033).  The result is
// update_nb_select()'s, on every lane.  False (r untouched) where update() runs its triangular
// stage (a grid-edge cell, or no valid square stencil): the caller then runs update_nb_select().
AF_DEV bool update_select_lanes(double tk, bool vk, AF_UPD_IDX iz, AF_UPD_IDX ix, AF_UPD_IDX nnz, AF_UPD_IDX nnx,
                                int lane, UpdSel& r) {
    using I = AF_UPD_IDX;
    if (ix == 0 || ix == nnx - 1 || iz == 0 || iz == nnz - 1) return false;
    // interior: every position of the 12 is inside the operator's bounds (update_nb_select's inb)
    const bool r2 = ix < nnx - 2, l2 = ix > 1, u2 = iz > 1, d2 = iz < nnz - 2;
    const unsigned inb = 2u | 4u | 32u | 64u | 256u | 512u | 1024u | 2048u | (l2 ? 1u : 0u) | (r2 ? 8u : 0u) |
                         (u2 ? 16u : 0u) | (d2 ? 128u : 0u);
    const unsigned em = (unsigned)__ballot(lane < 12 && vk) & inb;
    // slots of stencil k packed 4 bits per stencil: apex, a, b (update_nb_select's AP / SA / SB)
    constexpr unsigned kAP = nib8(4, 3, 7, 0, 8, 9, 11, 10), kSA = nib8(8, 9, 10, 8, 1, 5, 6, 1),
                       kSB = nib8(9, 11, 11, 10, 5, 2, 2, 6);
    const int k = lane & 7;
    const int sa = (int)((kSA >> (4 * k)) & 15u), sb = (int)((kSB >> (4 * k)) & 15u), ap = (int)((kAP >> (4 * k)) & 15u);
    const double ta = __shfl(tk, sa), tb = __shfl(tk, sb);
    const unsigned msk = (1u << ap) | (1u << sa) | (1u << sb);
    const double d = fabs(ta - tb);
    double key = (lane < 8 && (em & msk) == msk && d < 1000000.0) ? d : INFINITY;
    int idx = lane < 8 ? lane : 64;
#if AF_SEL_DPP
    // lanes 0..7: partners by DPP (quad xor 1, quad xor 2, half-row mirror), no LDS round trip
    auto step = [&](double ok, int oi) {
        if (ok < key || (ok == key && oi < idx)) {
            key = ok;
            idx = oi;
        }
    };
    step(dpp_d<0xB1>(key), dpp_i<0xB1>(idx));
    step(dpp_d<0x4E>(key), dpp_i<0x4E>(idx));
    step(dpp_d<0x141>(key), dpp_i<0x141>(idx));
#else
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
        const double ok = __shfl_xor(key, o);
        const int oi = __shfl_xor(idx, o);
        if (ok < key || (ok == key && oi < idx)) {
            key = ok;
            idx = oi;
        }
    }
#endif
    if (!(lane_d(key, 0) < INFINITY)) return false;
    const int sno = __builtin_amdgcn_readfirstlane(idx);
    const int pa_s = (int)((kSA >> (4 * sno)) & 15u), pb_s = (int)((kSB >> (4 * sno)) & 15u);
    const int p_s = (int)((kAP >> (4 * sno)) & 15u);
    const double yap = lane_d(tk, p_s), ya = lane_d(tk, pa_s), yb = lane_d(tk, pb_s);
    // slot -> (dz + 2) * 8 + (dx + 2), 6 bits per slot (update_nb_select's OFF)
    constexpr unsigned long long kOff = (16ull) | (17ull << 6) | (19ull << 12) | (20ull << 18) | (2ull << 24) |
                                        (10ull << 30) | (26ull << 36) | (34ull << 42) | (9ull << 48) |
                                        (11ull << 54);
    auto off = [&](int s) -> int { return s < 10 ? (int)((kOff >> (6 * s)) & 63ull) : (s == 10 ? 25 : 27); };
    const bool lo = ya < yb;
    const int p1 = off(p_s), p2 = off(lo ? pa_s : pb_s), p3 = off(lo ? pb_s : pa_s);
    r.w.x1 = ix + (p1 & 7) - 2;
    r.w.z1 = iz + (p1 >> 3) - 2;
    r.w.x2 = ix + (p2 & 7) - 2;
    r.w.z2 = iz + (p2 >> 3) - 2;
    r.w.x3 = ix + (p3 & 7) - 2;
    r.w.z3 = iz + (p3 >> 3) - 2;
    r.w.y1 = yap;
    r.w.y2 = lo ? ya : yb;
    r.w.y3 = lo ? yb : ya;
    r.w.have = true;
    r.wt = r.w.y2;
    r.angle = 0.0;
    r.dist = -1.0;
    (void)sizeof(I);
    return true;
}

// update()'s finish out of line (AF_FINISH_OOL 1, the init and exact-walk kernels): one copy of the
// wavefront-angle and phase-velocity code per kernel instead of one per call site (measured: init
// +1 %, subgrid-9 exact walk -1.5 %, profiles/r5t; off).  The arguments
// are scalars (32 VGPRs: none go through the stack); vp_nc = velpn | ncol << 16 (set_model keeps
// ncol below 2^15).  Same arithmetic as upd_finish.
#ifndef AF_FINISH_OOL
#define AF_FINISH_OOL 0
#endif
#if AF_FINISH_OOL
__attribute__((noinline))
#endif
AF_DEV double upd_finish_ool(const double* ptab, int vp_nc, double veln, double vm, const double* stif, int ix, int iz,
                             int x1, int x2, int x3, int z1, int z2, int z3, double y1, double y2, double y3, int have,
                             double wt, double angle, double dist, double dnx) {
    if (have) wad(ix, iz, x1, x2, x3, z1, z2, z3, y1, y2, y3, angle, dist);
    if (dist != -1.0) {
        const int velpn = vp_nc & 0xffff, ncol = vp_nc >> 16;
        double effa = pymod(veln - angle, 180);
        double velocity;
        if (velpn != 0 || stif == nullptr) velocity = table_vel(ptab, ncol, effa, velpn, vm);
        else velocity = christoffel_phase(stif, effa, vm);
        return wt + (dist * dnx / velocity);
    }
    return -1.0;
}

AF_DEV double update_nb_finish(const DevModel& M, const CellMat& cm, AF_UPD_IDX iz, AF_UPD_IDX ix, double dnx,
                               const UpdSel& r) {
    return upd_finish(M, cm, ix, iz, r.w, r.wt, r.angle, r.dist, dnx);
}
// the same through upd_finish_ool (int coordinates)
AF_DEV double update_nb_finish_ool(const DevModel& M, const CellMat& cm, int iz, int ix, double dnx, const UpdSel& r) {
    static_assert(std::is_same<AF_UPD_IDX, int>::value, "int stencil coordinates");
    return upd_finish_ool(M.ptab, cm.velpn | (M.ncol << 16), cm.veln, cm.vm, cm.stif, ix, iz, r.w.x1, r.w.x2, r.w.x3,
                          r.w.z1, r.w.z2, r.w.z3, r.w.y1, r.w.y2, r.w.y3, r.w.have ? 1 : 0, r.wt, r.angle, r.dist,
                          dnx);
}

template <class F>
AF_DEV double update_nb(const F& f, const DevModel& M, const CellMat& cm, AF_UPD_IDX iz, AF_UPD_IDX ix, double dnx,
                        AF_UPD_IDX nnz, AF_UPD_IDX nnx) {
    const UpdSel r = update_nb_select(f, iz, ix, nnz, nnx);
#ifdef AF_UPD_HOOK
    AF_UPD_HOOK(r.wt + r.angle + r.dist);  // profiling builds: the stencil stage is done
#endif
    return update_nb_finish(M, cm, iz, ix, dnx, r);
}

#ifndef AF_UPD_LEAN
#define AF_UPD_LEAN 1
#endif
template <class F, class = void>
struct upd_regs : std::false_type {};
template <class F>
struct upd_regs<F, std::void_t<decltype(&F::t11)>> : std::true_type {};

// update() (Anis_TTF_rays.py:904-1410): the branch-free form on register neighbourhoods, the
// reference form on every other field accessor
template <class F>
AF_DEV double update(const F& f, const DevModel& M, const CellMat& cm, AF_UPD_IDX iz, AF_UPD_IDX ix, double dnx,
                     AF_UPD_IDX nnz, AF_UPD_IDX nnx) {
    if constexpr (AF_UPD_LEAN && upd_regs<F>::value) return update_nb(f, M, cm, iz, ix, dnx, nnz, nnx);
    else return update_ref(f, M, cm, iz, ix, dnx, nnz, nnx);
}

}  // namespace af
