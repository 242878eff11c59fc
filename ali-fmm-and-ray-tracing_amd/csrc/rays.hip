// rays.hip — plane-search ray back-trace find_ray (Anis_TTF_rays.py:3104-3465) on gfx950.
//
// One group of G lanes per ray (G = 16, 32 or 64: the smallest power of two >= the 6*sg+3
// candidates of an axis plane, so subgrid 1 packs 4 rays into a wavefront; G = 64 loops over the
// candidates when there are more; G = 9 at subgrid 1 when the request fills the device with 7 rays
// per wavefront, af_ray_group_lanes).  Each step is uniform within the group except the candidate
// evaluation: lane i evaluates candidate i of the plane (6*sg+3 candidates on axis planes,
// <= 5*sg+3 on diagonal planes), i.e. rec_TTF at the candidate plus the straight-segment time
// time_between_points (:2835-2989, a DDA over coarse cells).  The parabolic local-minimum search
// (:3192-3218) is a lexicographic (value, order) reduction over the group's lanes, which selects
// exactly the candidate the reference's sequential strict-'<' scan selects.  ray_time (:2992-3022) is
// summed after the walk, the group's lanes evaluating consecutive segments and lane order giving
// the reference's left-to-right sum, so times match the CPU to the last bit (the trigonometry is
// correctly rounded, cr_math.h).  All arithmetic is double precision.
// Every candidate's time_between_points() is a chain of dependent reads (material id, material
// record, stiffness row or group table, the trig tables): with LDSMAT the records, stiffness rows,
// group table and the CR trig tables are staged in LDS once per workgroup, so only the material-id
// byte comes from memory.
#define CR_LDS_TABLES  // cr_math.h tables in LDS (crm::lds_init at kernel start)
#include <type_traits>
#include "kernels.h"

namespace af {



constexpr int kRayWaves = 4;
constexpr int kMaxCand = 256;
constexpr int kRayMatLds = 256, kRayStabLds = 64, kRayGtabLds = 722;

struct Key {
  double v;
  int order;
  double pos;
};
AF_DEV bool key_less(const Key& a, const Key& b) { return a.v < b.v || (a.v == b.v && a.order < b.order); }

// wavefronts per SIMD the kernel is compiled for (174 VGPRs at 2; 3 or 4 force fewer registers and
// measured no faster, profiles/r5q; the LDS of a 4-wavefront block also allows two blocks per CU)
#ifndef AF_RAY_WPE
#define AF_RAY_WPE 2
#endif
// Material runs: time_between_points() evaluates the group velocity once per run of pieces in one
// material; the lanes of a wavefront reach their runs' evaluations at different pieces, so the
// one-lane loop re-issues the evaluation for every piece index at which any lane changes material.
// tbp_wave walks every active lane's segment first (runs: material id and first piece; the piece
// lengths are kept in LDS), spreads the runs' evaluations over the active lanes (rounds of one
// evaluation per lane), then sums the pieces in the reference's order (segments longer than the
// kept pieces walk again).  The same values: a run's slowness depends on its material record and
// the segment's angle only.
#ifndef AF_RAY_BATCH
#define AF_RAY_BATCH 1
#endif
// material ids of a segment's first pieces read ahead of the run scan (0: one read per piece)
#ifndef AF_RAY_PF
#define AF_RAY_PF 8
#endif
constexpr int kRuns = 4;  // runs per segment handled this way (more: the one-lane loop)
// piece lengths kept from the first walk for the summing one (segments of more pieces walk again)
#ifndef AF_RAY_PC
#define AF_RAY_PC 12
#endif
constexpr int kPc = AF_RAY_PC;
struct RayScratch {  // per wavefront
  double slo[64 * kRuns];
  double ang[64];
  int item[64 * kRuns];
  double dist[64 * (kPc > 0 ? kPc : 1)];  // piece k of lane l: dist[64 k + l]
};

// the group-velocity evaluation, one copy in the kernel: inlined at every call site the kernel's
// code was 131 KB, out of line 18 + 27 KB at the same speed (profiles/r5q; AF_RAY_SLO_NOINLINE 0:
// inlined)
#ifndef AF_RAY_SLO_NOINLINE
#define AF_RAY_SLO_NOINLINE 1
#endif
#if AF_RAY_SLO_NOINLINE
__attribute__((noinline))
#endif
AF_DEV double ray_slowness(double veln, double vm, int velpn, const double* stif, double angle, const double* gtab,
                           int ncol) {
  // tbp_slowness / group_vel_cell with the record's fields
#ifdef AF_RAY_DIAG_SLO  // diagnostic build only (wrong rays): the kernel without the evaluations
  return 1.0 / (vm + 1e-9 * angle + 1e-12 * veln);
#endif
  const double eff = pymod(veln - angle, 180);
  const double velocity =
      (velpn != 0 || stif == nullptr) ? table_vel(gtab, ncol, eff, velpn, vm) : christoffel_group(stif, eff, vm);
  return 1.0 / velocity;
}
AF_DEV double ray_slowness(const DevModel& M, const MatLds& ms, int id, double angle) {
  const MatRec m = ms.mat[id];
  return ray_slowness(m.veln, m.vm, m.velpn, m.sidx >= 0 ? ms.stab + 5 * m.sidx : nullptr, angle, ms.gt, M.ncol);
}

AF_DEV double tbp_wave(const DevModel& M, const MatLds& ms, RayScratch& S, bool valid, double x1, double x2, double y1,
                       double y2, double dnx, int sg, int wl) {
  TbpWalk w;
  double angle = 0.0;
  unsigned ids = 0, starts = 0;  // run r: material id in byte r, first piece in byte r
  int nr = 0, npc = 0;            // runs, pieces
  if (valid) {
    w.setup(x1, x2, y1, y2, sg, angle);
    w.begin();
    int last = -1;
    auto run = [&](int k, int id) {
      if (id != last) {
        if (nr < kRuns && k < 256) {
          ids |= (unsigned)id << (8 * nr);
          starts |= (unsigned)k << (8 * nr);
        } else {
          nr = kRuns;  // (k >= 256: over as well)
        }
        nr++;
        last = id;
      }
    };
    int k = 0;
    if constexpr (AF_RAY_PF > 0) {
      // the first AF_RAY_PF pieces' material ids: reads issued together (the walk's geometry does
      // not depend on them), one memory latency instead of one per piece
      int idv[AF_RAY_PF > 0 ? AF_RAY_PF : 1];
      int npf = 0;
#pragma unroll
      for (int q = 0; q < AF_RAY_PF; q++) {
        idv[q] = 0;
        if (!w.done()) {
          double nxv, nyv;
          w.piece(nxv, nyv);
          int yp, xp;
          w.cell(M, nxv, nyv, yp, xp);
          idv[q] = ms.id(yp, xp);
          if (q < kPc) S.dist[64 * q + wl] = w.piece_dist(nxv, nyv, dnx);
          w.prev_x = nxv;
          w.prev_y = nyv;
          npf = q + 1;
        }
      }
#pragma unroll
      for (int q = 0; q < AF_RAY_PF; q++)
        if (q < npf) run(q, idv[q]);
      k = npf;
    }
    for (; !w.done(); k++) {  // the rest (long segments)
      double nxv, nyv;
      w.piece(nxv, nyv);
      int yp, xp;
      w.cell(M, nxv, nyv, yp, xp);
      run(k, ms.id(yp, xp));
      if (k < kPc) S.dist[64 * k + wl] = w.piece_dist(nxv, nyv, dnx);
      w.prev_x = nxv;
      w.prev_y = nyv;
    }
    npc = k;
  }
  // over: more runs than kRuns (rare): this lane evaluates its runs in the summing walk
  const bool over = nr > kRuns;
  const int nb = over ? 0 : nr;
  S.ang[wl] = angle;
  const unsigned long long lt = (1ull << wl) - 1ull;
  // the runs as items (lane, run, material id), compacted over the wavefront
  int ntot = 0;
#pragma unroll
  for (int r = 0; r < kRuns; r++) {
    const unsigned long long m = __ballot(nb > r);
    if (nb > r) S.item[ntot + __popcll(m & lt)] = (wl << 10) | (r << 8) | (int)((ids >> (8 * r)) & 255u);
    ntot += __popcll(m);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const unsigned long long act = __ballot(true);
  const int rank = __popcll(act & lt), nact = __popcll(act);
  for (int b = 0; b < ntot; b += nact) {
    const int j = b + rank;
    if (j < ntot) {
      const int it = S.item[j];
      const int l = it >> 10, r = (it >> 8) & 3, id = it & 255;
#ifdef AF_RAY_DIAG_DBL  // diagnostic build: every evaluation twice (its marginal cost), same results
      double a2 = S.ang[l];
      asm volatile("" : "+v"(a2));
      const double s2 = ray_slowness(M, ms, id, a2);
      S.slo[l * kRuns + r] = ray_slowness(M, ms, id, S.ang[l]) + (s2 == -12345.0 ? 1.0 : 0.0);
#else
      S.slo[l * kRuns + r] = ray_slowness(M, ms, id, S.ang[l]);
#endif
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (!valid) return 0.0;
  double section_time = 0.0;
  int r = 0, last = -1;
  double slown = over ? 0.0 : S.slo[wl * kRuns];
  int next_start = !over && nr > 1 ? (int)((starts >> 8) & 255u) : -1;
  if (!over && npc <= kPc) {  // the kept piece lengths, summed in order
    for (int k = 0; k < npc; k++) {
      if (k == next_start) {
        r++;
        slown = S.slo[wl * kRuns + r];
        next_start = r + 1 < nr ? (int)((starts >> (8 * (r + 1))) & 255u) : -1;
      }
      section_time += S.dist[64 * k + wl] * slown;
    }
    return section_time;
  }
  w.begin();
  for (int k = 0; !w.done(); k++) {
    double nxv, nyv;
    w.piece(nxv, nyv);
    if (over) {
      int yp, xp;
      w.cell(M, nxv, nyv, yp, xp);
      const int id = ms.id(yp, xp);
      if (id != last) {
        slown = ray_slowness(M, ms, id, angle);
        last = id;
      }
    } else if (k == next_start) {
      r++;
      slown = S.slo[wl * kRuns + r];
      next_start = r + 1 < nr ? (int)((starts >> (8 * (r + 1))) & 255u) : -1;
    }
    section_time += w.piece_time(nxv, nyv, dnx, slown);
    w.prev_x = nxv;
    w.prev_y = nyv;
  }
  return section_time;
}

template <int G, bool LDSMAT>
__global__ __launch_bounds__(64 * kRayWaves) __attribute__((amdgpu_waves_per_eu(AF_RAY_WPE))) void find_ray_kernel(
    RayParams P) {
  constexpr int kGroups = 64 / G;             // rays per wavefront
  constexpr int kTT = kMaxCand / kGroups;      // candidate slots per ray
  __shared__ double TTs[kRayWaves][kMaxCand];
  __shared__ double RTs[kRayWaves][kMaxCand];  // rec_TTF at the candidates (the step's new point reads it)
  __shared__ MatRec smat[LDSMAT ? kRayMatLds : 1];
  __shared__ double sstab[LDSMAT ? 5 * kRayStabLds : 1];
  __shared__ double sgtab[LDSMAT ? kRayGtabLds : 1];
  __shared__ RayScratch RS[LDSMAT && AF_RAY_BATCH ? kRayWaves : 1];
  crm::lds_init();
  if (LDSMAT) {
    for (int k = threadIdx.x; k < P.M.nmat; k += blockDim.x) smat[k] = P.M.mtab[k];
    for (int k = threadIdx.x; k < 5 * P.M.nstab; k += blockDim.x) sstab[k] = P.M.stab[k];
    for (int k = threadIdx.x; k < 361 * P.M.ncol; k += blockDim.x) sgtab[k] = P.M.gtab[k];
  }
  __syncthreads();
  const std::conditional_t<LDSMAT, MatLds, MatGlobal> ms = [&] {
    if constexpr (LDSMAT) return MatLds{P.M, smat, sstab, sgtab};
    else return MatGlobal{P.M};
  }();
  // a group of G lanes per ray: G a power of two, or 9 (subgrid 1: the 9 axis-plane candidates,
  // 7 rays per wavefront, lane 63 idle); gbase = the group's first lane in the wavefront
  constexpr bool kPow2 = (G & (G - 1)) == 0;
  const int wl = threadIdx.x & 63, w = threadIdx.x >> 6, grp = wl / G, lane = wl - grp * G, gbase = grp * G;
  const int ray = (blockIdx.x * kRayWaves + w) * kGroups + grp;
  if (grp >= kGroups || ray >= P.nrays) return;
  const RayJob J = P.jobs[ray];
  const int sg = P.sg;
  const int sd = 3 * sg + 1, sd2 = 2 * sg + 1;
  const int nnx = P.fnz, nnz = P.fnx;  // reference naming (:3151-3152)
  double* rxo = P.ray_x + (long)ray * P.max_pts;
  double* ryo = P.ray_y + (long)ray * P.max_pts;
  double* TT = &TTs[w][grp * kTT];
  double* RTc = &RTs[w][grp * kTT];
  long cap = 5L * (P.M.nz0 + P.M.nx0);
  if (cap > P.max_pts) cap = P.max_pts;
  const double recx = J.rx, recy = J.ry;
  double last_x = J.sx, last_y = J.sy;
  double lvx = recx - J.sx, lvy = recy - J.sy;
  long ray_len = 1;
  int flags = 0;
  double tt = 0.0;  // ray_time :2992-3022, accumulated segment by segment in the reference's order
  if (lane == 0) {
    rxo[0] = J.sx;
    ryo[0] = J.sy;
  }
#define RT(r, c) gld(J.ttf + (long)(r) * P.fnx + (long)(c))
  // rec_TTF at the rounded last point (:3406): carried from step to step
  double rt_last = RT(pyround_i(last_y), pyround_i(last_x));
  while ((last_x - recx) * (last_x - recx) + (last_y - recy) * (last_y - recy) > (1.6 * sg) * (1.6 * sg)) {
    if ((last_x - recx) * (last_x - recx) + (last_y - recy) * (last_y - recy) < (double)(4 * sg) * (4 * sg)) {
      lvx = recx - last_x;
      lvy = recy - last_y;
    }
    if (ray_len + 1 >= cap) {
      flags |= 2;
      break;
    }
    double cand[4] = {fabs(lvx), fabs(lvx + lvy) / sqrt(2.0), fabs(lvy), fabs(lvx - lvy) / sqrt(2.0)};
    int dir = 0;
    for (int q = 1; q < 4; q++)
      if (cand[q] > cand[dir]) dir = q;
    // grid coordinates in int (fields stay below 32768 nodes a side)
    int rlx = pyround_i(last_x), rly = pyround_i(last_y);
    int c_value = 0, base0 = 0, n = 0;
    bool stop = false;
    if (dir == 0) {
      c_value = rlx + (lvx > 0 ? sg : -sg);
      if (c_value < 0 || c_value >= nnz) stop = true;
      int mn = max(0, rly - sd), mx = min(nnx - 1, rly + sd);
      base0 = mn;
      n = mx - mn + 1;
    } else if (dir == 1) {
      c_value = rlx + rly;
      int mn, mx;
      if (lvx > 0) {
        c_value += sg;
        mn = max(max(0, c_value - (nnx - 1)), rlx - sd2);
        mx = min(min(nnz - 1, c_value), c_value - rly + sd2);
      } else {
        c_value -= sg;
        mn = max(max(0, c_value - (nnx - 1)), c_value - rly - sd2);
        mx = min(min(nnz - 1, c_value), rlx + sd2);
      }
      base0 = mn;
      n = mx - mn + 1;
    } else if (dir == 2) {
      c_value = rly + (lvy > 0 ? sg : -sg);
      if (c_value < 0 || c_value >= nnx) stop = true;
      int mn = max(0, rlx - sd), mx = min(nnz - 1, rlx + sd);
      base0 = mn;
      n = mx - mn + 1;
    } else {
      c_value = rly - rlx;
      int mn, mx;
      if (lvx < 0) {
        c_value += sg;
        mn = max(max(0, -c_value), rly - c_value - sd2);
        mx = min(min(nnz - 1, (nnx - 1) - c_value), rlx + sd2);
      } else {
        c_value -= sg;
        mn = max(max(0, -c_value), rlx - sd2);
        mx = min(min(nnz - 1, (nnx - 1) - c_value), rly - c_value + sd2);
      }
      base0 = mn;
      n = mx - mn + 1;
    }
    if (stop) break;
    if (n <= 0 || n > kTT) {
      flags |= 4;
      break;
    }
    // candidates across lanes
    for (int i0 = 0; i0 < n; i0 += G) {
      const int i = i0 + lane;
      const bool ok = i < n;
      // candidate i's grid point (column xa, row ya): rec_TTF there + the straight segment's time
      int xa, ya;
      if (dir == 0) {
        xa = c_value;
        ya = i + base0;
      } else if (dir == 1) {
        xa = base0 + i;
        ya = -xa + c_value;
      } else if (dir == 2) {
        xa = i + base0;
        ya = c_value;
      } else {
        xa = base0 + i;
        ya = xa + c_value;
      }
      const double rt = ok ? RT(ya, xa) : 0.0;
      double tb;
      if constexpr (LDSMAT && AF_RAY_BATCH) {
        tb = tbp_wave(P.M, ms, RS[w], ok, last_x, (double)xa, last_y, (double)ya, P.dnx, sg, wl);
      } else {
        tb = ok ? tbp(P.M, ms, last_x, (double)xa, last_y, (double)ya, P.dnx, sg) : 0.0;
      }
      if (ok) {
        TT[i] = rt + tb;
        RTc[i] = rt;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // local minima (:3192-3218): init key (order 0) + each strict parabola minimum (order j)
    Key best;
    if (TT[0] < TT[n - 1]) best = Key{TT[0], 0, 0.0};
    else best = Key{TT[n - 1], 0, (double)(n - 1)};
    for (int j0 = 1; j0 < n - 1; j0 += G) {
      int j = j0 + lane;
      if (j < n - 1) {
        double t1 = TT[j - 1], t2 = TT[j], t3 = TT[j + 1];
        if (t1 >= t2 && t2 <= t3) {
          double a = (t1 + t3 - 2 * t2) / 2;
          double b = (t3 - t1) / 2;
          double c = t2;
          double pos, lmv;
          if (a != 0) {
            pos = -b / (2 * a);
            lmv = a * (pos * pos) + b * pos + c;
            pos += (double)j;
          } else {
            pos = (double)j;
            lmv = t2;
          }
          Key k{lmv, (int)j, pos};
          if (key_less(k, best)) best = k;
        }
      }
    }
    if (kPow2) {
      for (int o = G / 2; o > 0; o >>= 1) {  // stays inside the aligned group of G lanes
        Key other{__shfl_xor(best.v, o), __shfl_xor(best.order, o), __shfl_xor(best.pos, o)};
        if (key_less(other, best)) best = other;
      }
    } else {
      // lane i takes lane i + o of its group (o = 1, 2, 4, 8): lane 0 ends with the group's
      // minimum (the order is total: the selection does not depend on the tree), then broadcasts
      for (int o = 1; o < G; o <<= 1) {
        const int src = lane + o < G ? wl + o : wl;
        Key other{__shfl(best.v, src), __shfl(best.order, src), __shfl(best.pos, src)};
        if (key_less(other, best)) best = other;
      }
      best = Key{__shfl(best.v, gbase), __shfl(best.order, gbase), __shfl(best.pos, gbase)};
    }
    const double min_i = best.pos;
    double nx_, ny_;
    if (dir == 0) {
      nx_ = (double)c_value;
      ny_ = min_i + (double)base0;
    } else if (dir == 1) {
      nx_ = (double)base0 + min_i;
      ny_ = (double)c_value - nx_;
    } else if (dir == 2) {
      nx_ = min_i + (double)base0;
      ny_ = (double)c_value;
    } else {
      nx_ = (double)base0 + min_i;
      ny_ = nx_ + (double)c_value;
    }
    // rec_TTF at the rounded new point: a candidate's (read in the candidate pass) when the point
    // rounds onto the search plane, which it does except at exact .5 ties on diagonal planes
    const int nrz = pyround_i(ny_), nrx = pyround_i(nx_);
    int ci = -1;
    if (dir == 0) ci = nrx == c_value ? nrz - base0 : -1;
    else if (dir == 2) ci = nrz == c_value ? nrx - base0 : -1;
    else if (dir == 1) ci = nrz == c_value - nrx ? nrx - base0 : -1;
    else ci = nrz == nrx + c_value ? nrx - base0 : -1;
    const double rt_new = (ci >= 0 && ci < n) ? RTc[ci] : RT(nrz, nrx);
    if (rt_last < rt_new) {
      flags |= 1;  // "Travel time to receiver increasing: Finishing ray early" (:3406-3407)
      break;
    }
    rt_last = rt_new;
    if (lane == 0) {
      rxo[ray_len] = nx_;
      ryo[ray_len] = ny_;
    }
    lvx = nx_ - last_x;
    last_x = nx_;
    lvy = ny_ - last_y;
    last_y = ny_;
    ray_len += 1;
    __builtin_amdgcn_wave_barrier();
  }
#undef RT
  if (lane == 0) {
    rxo[ray_len] = recx;
    ryo[ray_len] = recy;
  }
  const long npts = ray_len + 1;
  // ray_time (:2992-3022) after the walk: the group's lanes evaluate G segments at a time (each a
  // time_between_points() of consecutive points, read back from the ray buffer) and lane order
  // gives the reference's left-to-right sum, so the per-step walk carries no serial segment time
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");  // lane 0's point stores, visible to the group
#ifdef AF_RAY_DIAG_NOTIME  // diagnostic build only (no ray times): the walk alone
  for (long k0 = 0; k0 < 0; k0 += G) {
#else
  for (long k0 = 0; k0 < npts - 1; k0 += G) {
#endif
    const long k = k0 + lane;
    const bool ok = k < npts - 1;
    double seg = 0.0;
    if constexpr (LDSMAT && AF_RAY_BATCH) {
      const double xa = ok ? gld(rxo + k) : 0.0, xb = ok ? gld(rxo + k + 1) : 0.0;
      const double ya = ok ? gld(ryo + k) : 0.0, yb = ok ? gld(ryo + k + 1) : 0.0;
      seg = tbp_wave(P.M, ms, RS[w], ok, xa, xb, ya, yb, P.dnx, sg, wl);
    } else {
      if (ok) seg = tbp(P.M, ms, gld(rxo + k), gld(rxo + k + 1), gld(ryo + k), gld(ryo + k + 1), P.dnx, sg);
    }
    const int m = (int)min((long)G, npts - 1 - k0);
    for (int l = 0; l < m; l++) tt += kPow2 ? __shfl(seg, l, G) : __shfl(seg, gbase + l);
  }
  if (lane == 0) {
    P.times[ray] = tt;
    P.ray_len[ray] = (int)npts;
    P.flags[ray] = flags;
  }
}

}  // namespace af

namespace af {
// pack per-ray point slots into one interleaved (x, z) buffer at host-computed offsets
__global__ void pack_rays_kernel(const double* rx, const double* ry, const int* len, const long long* off, int max_pts,
                                 double* packed) {
  const int ray = blockIdx.x;
  const int n = len[ray];
  const long long o = off[ray];
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    packed[2 * (o + i)] = rx[(long)ray * max_pts + i];
    packed[2 * (o + i) + 1] = ry[(long)ray * max_pts + i];
  }
}
}  // namespace af

extern "C" hipError_t af_launch_pack_rays(const double* rx, const double* ry, const int* len, const long long* off,
                                          int nrays, int max_pts, double* packed, hipStream_t stream) {
  if (nrays <= 0) return hipSuccess;
  hipLaunchKernelGGL(af::pack_rays_kernel, dim3(nrays), dim3(256), 0, stream, rx, ry, len, off, max_pts, packed);
  return hipGetLastError();
}

extern "C" int af_ray_waves_per_simd() { return AF_RAY_WPE; }

// lanes per ray (a power of two): candidates of one search plane across lanes; AF_RAY_GMIN 8 puts
// 8 rays in a wavefront at subgrid 1 (9 axis-plane candidates then take two rounds)
// subgrid 1: groups of exactly the 9 candidates (1) instead of 16 lanes (0)
#ifndef AF_RAY_G9
#define AF_RAY_G9 1
#endif
#ifndef AF_RAY_GMIN
#define AF_RAY_GMIN 16
#endif
// packed: the launch has rays enough to fill the device at 7 rays per wavefront (9-lane groups at
// subgrid 1); else 16 lanes (4 rays per wavefront: twice the wavefronts for a smaller launch)
extern "C" int af_ray_group_lanes(int sg, int packed) {
  const int ncand = 6 * sg + 3;  // axis planes; diagonal planes have <= 5*sg+3
  if (AF_RAY_G9 && packed && ncand == 9) return 9;  // subgrid 1: 7 rays of 9 lanes per wavefront
  return ncand <= AF_RAY_GMIN ? AF_RAY_GMIN : ncand <= 16 ? 16 : ncand <= 32 ? 32 : 64;
}

extern "C" hipError_t af_launch_rays(const af::RayParams* P, hipStream_t stream) {
  const int G = P->glanes > 0 ? P->glanes : af_ray_group_lanes(P->sg, 0);
  if (G != 9 && G != 8 && G != 16 && G != 32 && G != 64) return hipErrorInvalidValue;
  const int per_block = af::kRayWaves * (64 / G);
  const dim3 grid((P->nrays + per_block - 1) / per_block), block(64 * af::kRayWaves);
  // material records, stiffness rows and the group table in LDS when they fit (the per-cell ids
  // index the records)
  const bool lds = P->M.mid && P->M.mtab && P->M.nmat <= af::kRayMatLds && P->M.nstab <= af::kRayStabLds &&
                   361 * P->M.ncol <= af::kRayGtabLds;
  if (G == 9) {
    if (lds) hipLaunchKernelGGL((af::find_ray_kernel<9, true>), grid, block, 0, stream, *P);
    else hipLaunchKernelGGL((af::find_ray_kernel<9, false>), grid, block, 0, stream, *P);
  } else if (G == 8) {
    if (lds) hipLaunchKernelGGL((af::find_ray_kernel<8, true>), grid, block, 0, stream, *P);
    else hipLaunchKernelGGL((af::find_ray_kernel<8, false>), grid, block, 0, stream, *P);
  } else if (G == 16) {
    if (lds) hipLaunchKernelGGL((af::find_ray_kernel<16, true>), grid, block, 0, stream, *P);
    else hipLaunchKernelGGL((af::find_ray_kernel<16, false>), grid, block, 0, stream, *P);
  } else if (G == 32) {
    if (lds) hipLaunchKernelGGL((af::find_ray_kernel<32, true>), grid, block, 0, stream, *P);
    else hipLaunchKernelGGL((af::find_ray_kernel<32, false>), grid, block, 0, stream, *P);
  } else {
    if (lds) hipLaunchKernelGGL((af::find_ray_kernel<64, true>), grid, block, 0, stream, *P);
    else hipLaunchKernelGGL((af::find_ray_kernel<64, false>), grid, block, 0, stream, *P);
  }
  return hipGetLastError();
}
