// fmm_init.hip — source initialisation of travel() (Anis_TTF_rays.py:1508-1993) on gfx950.
//
// One workgroup per source, two wavefronts.  The three refined stage grids (5x5 coarse window x27,
// 13x13 x9, 27x27 x3; <= 109x109 nodes) live entirely in LDS (154 KB of the CU's 160 KB) and
// are solved with the reference's own heap-ordered FMM: the heap (with its round-half-even parent,
// SURVEY B-D3), the stage-1 nnz=nnx1 quirk (:1645, padded reads) and the hand-over order are
// reproduced exactly, so the init region is the reference's up to device transcendental ulps.
// The heap walk is inherently serial: wavefront 0 runs the heap (its sifts on one lane, a pop's
// neighbour classification on four), wavefront 1 relaxes each pop's neighbours while the heap
// runs downtree, and the next pop is handed over before the current pop's last sift-up when that
// sift-up cannot reach the root (stage_loop); all lanes clear LDS, fill the straight-ray footprint
// and decimate between stages.  Output: the decimated
// stage-3 nodes that the band kernel hands over to the main grid (:2006-2040), as (cell, ttn,
// class) triples.
#define CR_LDS_TABLES  // cr_math.h tables in LDS (crm::lds_init at kernel start)
#include "device_common.h"
#include "local_ops.h"
#include "kernels.h"
#include "fields.h"

namespace af {

constexpr int kInitMaxN = 109 * 109;  // largest stage grid (stage 1 / 2)
constexpr int kInitHeap = 1024;       // heap slots (the stage fronts stay below ~500 nodes)
constexpr int kInitMat = 256;         // material records staged in LDS (DevModel::mtab)
constexpr int kInitDec = 37 * 37;     // decimated stage-1/2 grid
constexpr int kInitWin = 53 * 53;     // coarse cells under a stage grid / the prefix window
constexpr int kInitStab = 64;         // stiffness rows staged in LDS
// diagnostic build (AF_INIT_DIAG=1): shader-clock cycles of the walk's activities, summed over the
// stages into prof[8..15] (heap: wait for relaxations, downtree, add/upd, classify; relax: wait
// for a pop, verification passes, evaluation passes, verification-pass count)
#ifndef AF_INIT_DIAG
#define AF_INIT_DIAG 0
#endif
// the heap role runs on its whole wavefront: the pop's neighbour classification spread over the
// lanes (AF_INIT_PARCLS; 0: one lane's loops).  Its sift-ups and downtree stay one lane's loops:
// lane-parallel versions (the ancestors / the min-child path read in one LDS round trip, ballot
// and readlane chains) and stores deferred to the end of a sift measured slower (profiles/r5d,
// profiles/r5i_init_deferred_stores_not_kept.txt)
#ifndef AF_INIT_PARCLS
#define AF_INIT_PARCLS 1
#endif
// the next pop classified and handed to the relax role before the last sift-up of the current
// one when that sift-up cannot reach the root (stage walks)
#ifndef AF_INIT_IPARENT
#define AF_INIT_IPARENT 1
#endif
#ifndef AF_INIT_EARLY
#define AF_INIT_EARLY 1
#endif
#if AF_INIT_DIAG
#define AF_DG_T0(v) const long long v = clock64();
#define AF_DG_ADD(L, k, v) (L)->dg[k] += clock64() - (v);
#define AF_DG_CNT(L, k) (L)->dg[k] += 1;
#else
#define AF_DG_CNT(L, k)
#define AF_DG_T0(v)
#define AF_DG_ADD(L, k, v)
#endif

struct InitLds {
  double T[kInitMaxN];
  double decT[kInitDec];
  short S[kInitMaxN];
  double hkey[kInitHeap];          // heap keys: ttn of the node (kept equal to it by add/upd)
  MatRec mat[kInitMat];
  double stab[5 * kInitStab];       // DevModel::stab (nstab <= kInitStab)
  unsigned short hcell[kInitHeap];  // heap nodes (z << 8) | x
  unsigned short dup[8];            // Heap: nodes with two heap entries (in LDS, not in the Heap
                                    // object: a dynamically indexed member would put the whole heap
                                    // state, LDS pointer included, in scratch -> flat LDS accesses)
  unsigned char smid[kInitWin];     // material ids of the coarse cells under the current grid
  signed char decC[kInitDec];       // 0 far, 1 known inner, 2 known outer, 3 close
  // heap role -> relax role hand-off of one pop's neighbours (two-wavefront heap walk)
  int cmd, done;                    // sequence numbers (cmd -1: stop)
  int njob;
  alignas(16) int job[4];           // packed (job_pack): node, kind 1 add (far), 2 upd (close), +4: stage-1 quirk nnz
  long long rbusy;                  // profile: relax-role ticks of the current walk
  long long rjobs;                  // profile: relaxations | fouds18_A() fallbacks << 32
#if AF_INIT_DIAG
  long long dg[12];                 // diagnostic build: shader-clock cycles per activity (AF_DG)
#endif
};

struct LdsField {
  const double* T;
  const short* S;
  int nz, nx;
  AF_DEV int st(long z, long x) const { return z >= nz ? -1 : (int)S[z * nx + x]; }
  AF_DEV double tt(long z, long x) const { return z >= nz ? 0.0 : T[z * nx + x]; }
};

// addtree / updtree / downtree (:94-237).  Keys are stored in the heap next to the node (a copy
// of its ttn, refreshed by every add/upd), so a sift level is one LDS read instead of two
// dependent ones; comparisons are exactly the reference's.  The reference compares live ttn, so
// a node with two heap entries (the stage-1 window corners, added by two of the edge loops
// :1601-1612) has both entries' keys change when its ttn does: such nodes are recorded (dup) and
// every key of theirs is refreshed with their ttn (sync).
constexpr int kInitDup = 8;
struct Heap {
  InitLds* L;
  int nz, nx;
  int ntr;
  int err;
  int ndup = 0;
  int pops = 0;
  AF_DEV int bz(int k) const { return L->hcell[k] >> 8; }
  AF_DEV int bx(int k) const { return L->hcell[k] & 255; }
  AF_DEV double tb(int k) const { return L->hkey[k]; }
  // round(t / 2), half-even (:123), in integer arithmetic (AF_INIT_IPARENT; 0: through a double)
  AF_DEV static int parent(int t) {
    if (!AF_INIT_IPARENT) return (int)rint((double)t / 2.0);
    const int m = t >> 1;
    return (t & 1) ? m + (m & 1) : m;
  }
  AF_DEV void sift(int iz, int ix, int tpc) { sift_up(iz, ix, tpc); }
  // The moving entry stays in registers while it sifts: one round of LDS reads per level (the
  // other entry's key and node), the status writes in the reference's order.
  AF_DEV void sift_up(int iz, int ix, int tpc) {
    const unsigned short mc = (unsigned short)((iz << 8) | ix);
    const double tv = L->hkey[tpc];
    int tpp = parent(tpc);
    while (tpp > 0) {
      const double kp = L->hkey[tpp];
      const unsigned short cp = L->hcell[tpp];
      if (!(tv < kp)) break;
      L->S[iz * nx + ix] = (short)tpp;
      L->S[(cp >> 8) * nx + (cp & 255)] = (short)tpc;
      L->hcell[tpc] = cp;
      L->hkey[tpc] = kp;
      tpc = tpp;
      tpp = parent(tpc);
    }
    L->hcell[tpc] = mc;
    L->hkey[tpc] = tv;
  }
  // addtree :94-138
  // fresh: the node is known to be far (a relaxation job; its status already reads 1, set by
  // the relax role), else its status tells whether it already has an entry
  AF_DEV void add(int iz, int ix, bool fresh = false) { add_key(iz, ix, L->T[iz * nx + ix], fresh); }
  // the same with the node's ttn given (read when its relaxation was posted)
  AF_DEV void add_key(int iz, int ix, double key, bool fresh) {
    ntr += 1;
    if (ntr >= kInitHeap) { err = 1; ntr = kInitHeap - 1; return; }
    if (!fresh && L->S[iz * nx + ix] > 0) {  // already in the heap: a second entry
      if (ndup == kInitDup) { err = 1; return; }
      L->dup[ndup++] = (unsigned short)((iz << 8) | ix);
    }
    L->S[iz * nx + ix] = (short)ntr;
    L->hcell[ntr] = (unsigned short)((iz << 8) | ix);
    L->hkey[ntr] = key;
    sift(iz, ix, ntr);
  }
  // updtree :141-175
  AF_DEV void upd(int iz, int ix) { upd_key(iz, ix, L->T[iz * nx + ix]); }
  AF_DEV void upd_key(int iz, int ix, double key) {
    const int tpc = L->S[iz * nx + ix];
    L->hkey[tpc] = key;
    sift(iz, ix, tpc);
  }
  // a node's ttn changed: every heap entry of a node with two entries takes the new value
  AF_DEV void sync(int iz, int ix) {
    const unsigned short c = (unsigned short)((iz << 8) | ix);
    bool d = false;
    for (int k = 0; k < ndup; k++) d |= L->dup[k] == c;
    if (!d) return;
    const double t = L->T[iz * nx + ix];
    for (int k = 1; k <= ntr; k++)
      if (L->hcell[k] == c) L->hkey[k] = t;
  }
  AF_DEV void pop_down() { down(); }
  // downtree :178-237 (the moving entry in registers, as in sift_up)
  AF_DEV void down() {
    if (ntr == 1) { ntr -= 1; return; }
    const unsigned short mc = L->hcell[ntr];
    const double km = L->hkey[ntr];
    const int ms = (mc >> 8) * nx + (mc & 255);
    L->S[ms] = 1;
    ntr -= 1;
    int tpp = 1, tpc = 2;
    while (tpc < ntr) {
      const double k1 = L->hkey[tpc], k2 = L->hkey[tpc + 1];
      const unsigned short c1 = L->hcell[tpc], c2 = L->hcell[tpc + 1];
      const bool right = k1 > k2;
      const int t = right ? tpc + 1 : tpc;
      const double kc = right ? k2 : k1;
      const unsigned short cc = right ? c2 : c1;
      if (kc < km) {
        L->S[ms] = (short)t;
        L->S[(cc >> 8) * nx + (cc & 255)] = (short)tpp;
        L->hcell[tpp] = cc;
        L->hkey[tpp] = kc;
        tpp = t;
        tpc = 2 * tpp;
      } else {
        tpc = ntr + 1;
      }
    }
    if (tpc == ntr) {
      const double kc = L->hkey[tpc];
      const unsigned short cc = L->hcell[tpc];
      if (kc < km) {
        L->S[ms] = (short)tpc;
        L->S[(cc >> 8) * nx + (cc & 255)] = (short)tpp;
        L->hcell[tpp] = cc;
        L->hkey[tpp] = kc;
        tpp = tpc;
      }
    }
    L->hcell[tpp] = mc;
    L->hkey[tpp] = km;
  }
};

// coarse cells under the current grid: rows cz0.., columns cx0.. (w per row); their material
// ids are in InitLds::smid (LDSMAT)
struct MidWin {
  int cz0, cx0, w, h;
};

// all lanes: the material ids of window W into LDS
AF_DEV void load_smid(const DevModel& M, InitLds* L, const MidWin& W, int lane, int nl) {
  for (int k = lane; k < W.w * W.h; k += nl) {
    const long c = (long)(W.cz0 + k / W.w) * M.nx0 + W.cx0 + k % W.w;
    L->smid[k] = M.mid8 ? gld(M.mid8 + c) : (unsigned char)gld(M.mid + c);
  }
}

// material of a node: the LDS id + the LDS record (LDSMAT), else the model arrays; *pre: the
// material's fouds18_A() slownesses (DevModel::mslo) or null
template <bool LDSMAT>
AF_DEV CellMat init_mat(const DevModel& M, const InitLds* L, const MatView& v, const MidWin& W, int z, int x,
                        const double** pre) {
  if (!LDSMAT) {
    *pre = nullptr;
    return cell_mat(M, v, z, x);
  }
  const int fz = v.lo1z + (z + v.side1z) / v.s1z, fx = v.lo1x + (x + v.side1x) / v.s1x;
  const int cz = v.lo2z + (fz + v.side2) / v.s2, cx = v.lo2x + (fx + v.side2) / v.s2;
  // W.w == 0: the window is larger than InitLds::smid (exact_r > 20), ids from the model
  const long gc = (long)cz * M.nx0 + cx;
  const int id = W.w ? (int)L->smid[(cz - W.cz0) * W.w + (cx - W.cx0)]
                     : (M.mid8 ? (int)gld(M.mid8 + gc) : gld(M.mid + gc));
  const MatRec m = L->mat[id];
  CellMat r;
  r.velpn = m.velpn;
  r.veln = v.quant ? (double)(int)m.veln : m.veln;
  r.vm = v.quant ? (double)(float)m.vm : m.vm;
  r.stif = m.sidx >= 0 ? M.stab + 5 * m.sidx : nullptr;
  *pre = M.mslo ? M.mslo + 8 * id + 4 * (v.quant ? 1 : 0) : nullptr;
  return r;
}

struct StageCfg {
  double dnx;
  int isx, isz, max_dist, quirk;
  MatView mv;
  MidWin mw;
};

// field accessor of the exact main-loop prefix: main-grid coordinates, LDS window storage;
// nodes outside the window have never been touched (far: nsts -1, ttn 0)
struct WinField {
  const double* T;
  const short* S;
  int wz0, wx0, wz1, wx1, ww;
  AF_DEV int st(long z, long x) const {
    return (z < wz0 || z > wz1 || x < wx0 || x > wx1) ? -1 : (int)S[(z - wz0) * ww + (x - wx0)];
  }
  AF_DEV double tt(long z, long x) const {
    return (z < wz0 || z > wz1 || x < wx0 || x > wx1) ? 0.0 : T[(z - wz0) * ww + (x - wx0)];
  }
};

// fouds18_A() (:240-901) on an LDS window: the relaxation's fallback when update() finds no stencil
AF_DEV double fouds18_win(const WinField& F, const DevModel& M, const CellMat& cm, int iz, int ix, double dnx,
                          double dnz, int nnx, int nnz, const double* pre) {
  return fouds18(F, M, cm, iz, ix, dnx, dnz, nnx, nnz, pre);
}


// Two-wavefront heap walk.  The reference relaxes a popped node's neighbours after downtree, and
// neither depends on the other: downtree only moves heap entries (keys and the positive heap
// indices in S), while update()/fouds18_A() read T and the validity / known-ness of S.  So lane 0
// of wavefront 0 (heap role) pops, classifies the neighbours in the reference's order and runs
// downtree, while lane 0 of wavefront 1 (relax role) relaxes them in that order; the heap role
// then performs their addtree / updtree in order.  A far neighbour is marked valid (S = 1) right
// after its relaxation, as the reference's addtree would before the next neighbour is relaxed.
// Same results as the one-lane walk, with downtree off the critical path.
constexpr int kJobAdd = 1, kJobUpd = 2, kJobQuirk = 4;
// packed relaxation job: LDS-local node z << 8 | x, kind << 16
AF_DEV int job_z(int j) { return (j >> 8) & 255; }
AF_DEV int job_x(int j) { return j & 255; }
AF_DEV int job_kind(int j) { return j >> 16; }
AF_DEV int job_pack(int z, int x, int kind) { return (z << 8) | x | (kind << 16); }
AF_DEV void post(int* w, int v) { __hip_atomic_store(w, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); }
// the waiting role backs off between polls (s_sleep) so that it does not take issue slots and
// LDS cycles from the working one
// the relax role's re-check of a changed speculative entry: lane-parallel stencil stage (1) or
// one lane (0)
#ifndef AF_INIT_PARSEL
#define AF_INIT_PARSEL 1
#endif
#ifndef AF_INIT_SLEEP
#define AF_INIT_SLEEP 1
#endif
AF_DEV bool await_value(int* w, int v) {  // false: timeout (the other role is gone)
  for (long spins = 0; __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != v; spins++) {
    if (AF_INIT_SLEEP) __builtin_amdgcn_s_sleep(AF_INIT_SLEEP);
    if (spins > (1L << 28)) return false;
  }
  return true;
}
AF_DEV bool await_at_least(int* w, int v) {  // false: timeout
  for (long spins = 0; __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v; spins++) {
    if (AF_INIT_SLEEP) __builtin_amdgcn_s_sleep(AF_INIT_SLEEP);
    if (spins > (1L << 28)) return false;
  }
  return true;
}
AF_DEV int await_change(int* w, int last) {  // the next value != last, or -2 on timeout
  for (long spins = 0;; spins++) {
    const int v = __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (v != last) return v;
    if (AF_INIT_SLEEP) __builtin_amdgcn_s_sleep(AF_INIT_SLEEP);
    if (spins > (1L << 28)) return -2;
  }
}

// heap role, one pop: hand the classified neighbours to the relax role, downtree, then each
// neighbour's addtree / updtree as soon as its relaxation is done (L->done counts relaxations), so
// the sift-ups run beside the later neighbours' relaxations (they only move heap indices: the
// validity the relaxations read stays).  false: the relax role timed out
// posted: the pop's jobs were already handed over (classified early, below).  early(key, cell):
// called before the last job's addtree / updtree with that node's new key and cell; it may
// classify the next pop and hand its jobs over first (they overwrite L->job: the job is read
// before), so that the relax role starts on them while this sift-up runs
template <class Early>
AF_DEV bool pop_two_role(Heap& h, int& seq, int& jobs, int n, bool posted, Early early) {
  InitLds* L = h.L;
  h.pops++;
  if (n == 0) {  // nothing to relax
    h.pop_down();
    return true;
  }
  if (!posted) {
    L->njob = n;
    post(&L->cmd, ++seq);
  }
  AF_DG_T0(td)
  h.pop_down();
  AF_DG_ADD(L, 1, td)
  for (int k = 0; k < n; k++) {
    AF_DG_T0(tw)
    if (!await_at_least(&L->done, jobs + k + 1)) return false;
    AF_DG_ADD(L, 0, tw)
    AF_DG_T0(ta)
    const int jk = L->job[k];
    const int jz = job_z(jk), jx = job_x(jk);
    const double key = L->T[jz * h.nx + jx];
    if (k == n - 1) early(key, (jz << 8) | jx);
    if (job_kind(jk) & kJobAdd) h.add_key(jz, jx, key, true);
    else h.upd_key(jz, jx, key);
    if (h.ndup) h.sync(jz, jx);
    AF_DG_ADD(L, 2, ta)
  }
  jobs += n;
  return true;
}
AF_DEV bool pop_two_role(Heap& h, int& seq, int& jobs, int n) {
  return pop_two_role(h, seq, jobs, n, false, [](double, int) {});
}

struct RelaxWin {
  int z0, x0, z1, x1, w;  // LDS window: rows z0..z1, columns x0..x1 (stage grids: the whole grid)
  int oz, ox;             // job coordinates (LDS-local) + (oz, ox) = operator coordinates
  int nnz, nnx;           // operator bounds
  double dnx, dnz;
  int quirk_nnz;          // update()'s nnz for quirk jobs (stage 1: nnx1, :1645)
  int has_quirk;          // this walk has quirk jobs (close x-neighbours in stage 1)
};

// v of lane l (l wave-uniform)
AF_DEV double readlane_d(double v, int l) { return lane_d(v, l); }

// lane k < 12: NbField slot k of (iz, ix) on an LDS grid (rows z0..z1, columns x0..x1, pitch w),
// the value and validity NbFieldT::load_lds gives that slot; other lanes: (0, false)
AF_DEV void lane_slot_lds(const double* T, const short* S, int z0, int x0, int z1, int x1, int w, int iz, int ix,
                          int lane, double& t, bool& v) {
  // (dz + 2) and (dx + 2) of slots 0..11, 4 bits each (NbFieldT::load_lds's order)
  constexpr unsigned long long kDZ = nib12(2, 2, 2, 2, 0, 1, 3, 4, 1, 1, 3, 3);
  constexpr unsigned long long kDX = nib12(0, 1, 3, 4, 2, 2, 2, 2, 1, 3, 1, 3);
  const int k = lane < 12 ? lane : 0;
  const int zz = iz + (int)((kDZ >> (4 * k)) & 15ull) - 2, xx = ix + (int)((kDX >> (4 * k)) & 15ull) - 2;
  const bool in = lane < 12 && zz >= z0 && zz <= z1 && xx >= x0 && xx <= x1;
  const int c = in ? (zz - z0) * w + (xx - x0) : 0;
  const double tv = T[c];
  const int sv = S[c];
  t = in ? tv : 0.0;
  v = in && sv >= 0;
}

// The relax role (wavefront 1).  A pop's neighbours are relaxed in order, each seeing the earlier
// ones' new values (the reference's sequence).  Relaxations are evaluated ahead of their turn, 64 at
// a time: when a job has no speculative entry, the whole wavefront runs one pass in which lane 0
// evaluates that job and every other lane a neighbour of one of the heap's first 16 entries (the
// next pops), against the current state; each lane keeps its result (node, value, update()'s
// stencil stage, the bounds mode it ran with) in registers, and a dirty flag that every committed
// relaxation sets when its node lies in the entry's 12-point stencil (only relaxations change T
// and validity: pops and sift-ups do not).  A job whose node has a clean entry takes the entry's
// value as it is; a dirty entry re-runs the cheap stencil stage on the state of its turn — equal
// to the entry's, the entry's value is the job's value (update()'s value is a function of its
// stencil stage's outputs), else the finish runs on that lane — so the results are the sequential
// ones bit for bit.  fouds18_A() (no usable stencil) always runs in turn.  The heap may be
// mid-sift while the lanes read it: any node read there is only a guess, never trusted.  (Round 3's
// relax role also predicted the next pop and verified its jobs ahead: the same speed, more code.)
template <bool LDSMAT>
AF_DEV void relax_role(InitLds* L, const DevModel& M, const MatView& mv, const MidWin& mw, const RelaxWin& R,
                          int lane) {
  int last = 0;
  long long busy = 0, njobs = 0, nf18 = 0, nburst = 0;
  const int wz = R.z1 - R.z0, wx = R.x1 - R.x0;
  int my_cell = -1, my_nnz = 0;
  bool my_dirty = true;
  double my_val = 0.0;
  UpdSel my_sel{};
  while (true) {
    int cmd = 0;
    AF_DG_T0(tcw)
    if (lane == 0) cmd = await_change(&L->cmd, last);
    if (lane == 0) { AF_DG_ADD(L, 4, tcw) }
    cmd = __shfl(cmd, 0);
    if (cmd < 0) break;
    last = cmd;
    const long long t0 = wall_clock64();
    const int nj = L->njob;
    const int4 jv = *reinterpret_cast<const int4*>(L->job);
    for (int k = 0; k < nj; k++) {
      AF_DG_T0(tv)
      const int jk = k == 0 ? jv.x : k == 1 ? jv.y : k == 2 ? jv.z : jv.w;
      const int lz = job_z(jk), lx = job_x(jk), kind = job_kind(jk);
      const int iz = lz + R.oz, ix = lx + R.ox;
      const int qnnz = (kind & kJobQuirk) ? R.quirk_nnz : R.nnz;
      const unsigned long long hm = __ballot(my_cell == (jk & 0xffff));
      double v;
      if (hm) {
        const int e = __ffsll((long long)hm) - 1;
        // a changed stencil (or bounds mode): the stage again, on the state of this turn — spread
        // over the wavefront (lanes 0..11 load a slot each, lanes 0..7 a square stencil each);
        // on one lane where update() runs its triangular stage
        if (__builtin_amdgcn_readlane((int)(my_dirty || my_nnz != qnnz), e)) {
          AF_DG_T0(trc)
          double tk;
          bool vk;
          lane_slot_lds(L->T, L->S, R.z0, R.x0, R.z1, R.x1, R.w, iz, ix, lane, tk, vk);
          UpdSel s2;
          const bool par = AF_INIT_PARSEL && update_select_lanes(tk, vk, iz, ix, qnnz, R.nnx, lane, s2);
          if (lane == e) {
            if (!par) {
              NbFieldT nb;
              nb.load_lds(L->T, L->S, R.z0, R.x0, R.z1, R.x1, R.w, iz, ix);
              s2 = update_nb_select(nb, iz, ix, qnnz, R.nnx);
            }
            if (!s2.same(my_sel)) {
              const double* pre;
              const CellMat cm = init_mat<LDSMAT>(M, L, mv, mw, iz, ix, &pre);
              my_val = update_nb_finish_ool(M, cm, iz, ix, R.dnx, s2);
              my_sel = s2;
            }
            my_dirty = false;
            my_nnz = qnnz;
          }
          if (lane == 0) {
            AF_DG_ADD(L, 7, trc)
            AF_DG_CNT(L, 8)
            if (!par) { AF_DG_CNT(L, 10) }
          }
        } else if (lane == 0) {
          AF_DG_CNT(L, 9)
        }
        v = readlane_d(my_val, e);
        if (lane == 0) { AF_DG_ADD(L, 5, tv) }
      } else {  // one pass: this job on lane 0, guesses of the next pops' jobs on the others
        int cz = lz, cx = lx, cnnz = qnnz;
        bool cand = true;
        if (lane > 0) {
          const int p = 1 + ((lane - 1) >> 2), d = (lane - 1) & 3;
          const int hc = L->hcell[p];
          cz = (hc >> 8) + (d == 2 ? -1 : d == 3 ? 1 : 0);
          cx = (hc & 255) + (d == 0 ? -1 : d == 1 ? 1 : 0);
          cand = cz >= 0 && cz <= wz && cx >= 0 && cx <= wx;
          const int st = cand ? (int)L->S[cz * R.w + cx] : 0;
          cand = cand && st != 0;
          cnnz = (R.has_quirk && d < 2 && st > 0) ? R.quirk_nnz : R.nnz;
        }
        if (cand) {
          const int gz = cz + R.oz, gx = cx + R.ox;
          const double* pre;
          const CellMat cm = init_mat<LDSMAT>(M, L, mv, mw, gz, gx, &pre);
          NbFieldT nb;
          nb.load_lds(L->T, L->S, R.z0, R.x0, R.z1, R.x1, R.w, gz, gx);
          my_sel = update_nb_select(nb, gz, gx, cnnz, R.nnx);
          my_val = update_nb_finish_ool(M, cm, gz, gx, R.dnx, my_sel);
          my_cell = (cz << 8) | cx;
          my_dirty = false;
          my_nnz = cnnz;
        } else {
          my_cell = -1;
        }
        nburst++;
        v = readlane_d(my_val, 0);
        if (lane == 0) { AF_DG_ADD(L, 6, tv) }
      }
      if (lane == 0) {
        if (v == -1.0) {
          const double* pre;
          const CellMat cm = init_mat<LDSMAT>(M, L, mv, mw, iz, ix, &pre);
          const WinField F{L->T, L->S, R.z0, R.x0, R.z1, R.x1, R.w};
          v = fouds18_win(F, M, cm, iz, ix, R.dnx, R.dnz, R.nnx, R.nnz, pre);
          nf18++;
        }
        L->T[lz * R.w + lx] = v;
        if (kind & kJobAdd) L->S[lz * R.w + lx] = 1;  // valid for the next relaxations (addtree sets the index)
        post(&L->done, (int)(njobs + 1));
      }
      if (my_cell >= 0) {  // the committed node changes the stencils that hold it
        const int dz = lz - (my_cell >> 8), dx = lx - (my_cell & 255), ad = abs(dz) + abs(dx);
        if (ad >= 1 && ad <= 2 && !(dz != 0 && dx != 0 && (abs(dz) != 1 || abs(dx) != 1))) my_dirty = true;
      }
      njobs++;
    }
    busy += wall_clock64() - t0;
  }
  if (lane == 0) {
    L->rbusy = busy;
    L->rjobs = njobs | (nburst << 24) | (nf18 << 44);
  }
}

// stage FMM loop (:1620-1674) over the two roles (tid 0: heap, wavefront 1: relax)
template <bool LDSMAT>
AF_DEV void stage_loop(Heap& h, const DevModel& M, const StageCfg& c, int tid) {
  InitLds* L = h.L;
  const int nz = h.nz, nx = h.nx;
  if (tid < 64) {  // heap role: wavefront 0 (uniform; single stores by lane 0)
    int seq = 0, jobs = 0;
    bool finished = false;
    // the root pop's classification: marks it known, writes its jobs, returns their number;
    // fin: a neighbour lies past the stage's max distance
    auto classify = [&](bool& fin) -> int {
      const int ix = h.bx(1), iz = h.bz(1);
      if (tid == 0) L->S[iz * nx + ix] = 0;
      int n = 0;
      bool finished = false;
      if (AF_INIT_PARCLS) {
        // lane d < 4: neighbour d in the reference's order (x - 1, x + 1, z - 1, z + 1)
        const int d = tid & 3;
        const int zz = d < 2 ? iz : (d == 2 ? iz - 1 : iz + 1), xx = d < 2 ? (d == 0 ? ix - 1 : ix + 1) : ix;
        const bool inb = tid < 4 && (d < 2 ? (0 <= xx && xx <= nx - 1) : (0 <= zz && zz <= nz - 1));
        const int st = inb ? (int)L->S[zz * nx + xx] : 0;
        const bool job = inb && (st == -1 || st > 0);
        const bool out = tid < 4 && !inb && (d < 2 ? abs(c.isx - xx) : abs(c.isz - zz)) == c.max_dist + 1;
        const unsigned long long jm = __ballot(job);
        if (__ballot(out)) finished = true;
        if (job)
          L->job[__popcll(jm & ((1ull << tid) - 1ull))] =
              job_pack(zz, xx, st == -1 ? kJobAdd : (kJobUpd | (d < 2 && c.quirk ? kJobQuirk : 0)));
        n = __popcll(jm);
      } else {
        for (int s = 0; s < 2; s++) {
          const int i = s == 0 ? ix - 1 : ix + 1;
          if (0 <= i && i <= nx - 1) {
            const int st = L->S[iz * nx + i];
            if (st == -1 || st > 0) {
              L->job[n] = job_pack(iz, i, st == -1 ? kJobAdd : (kJobUpd | (c.quirk ? kJobQuirk : 0)));
              n++;
            }
          } else if (abs(c.isx - i) == c.max_dist + 1) {
            finished = true;
          }
        }
        for (int s = 0; s < 2; s++) {
          const int i = s == 0 ? iz - 1 : iz + 1;
          if (0 <= i && i <= nz - 1) {
            const int st = L->S[i * nx + ix];
            if (st == -1 || st > 0) {
              L->job[n] = job_pack(i, ix, st == -1 ? kJobAdd : kJobUpd);
              n++;
            }
          } else if (abs(c.isz - i) == c.max_dist + 1) {
            finished = true;
          }
        }
      }
      fin = finished;
      return n;
    };
    // a pop classified (and its jobs handed over) while the previous pop's last sift-up was due
    int pre_n = -1;
    bool pre_fin = false;
    while (h.ntr > 0 && !finished && !h.err) {
      AF_DG_T0(tc)
      int n;
      const bool posted = pre_n >= 0;
      if (posted) {
        n = pre_n;
        finished = pre_fin;
        pre_n = -1;
      } else {
        n = classify(finished);
      }
      AF_DG_ADD(L, 3, tc)
      // the next pop is known before the last job's sift-up when that job can neither reach the
      // root (its key is not below the root's: sift-ups move on strict '<') nor be the root, and no
      // node has two heap entries (their keys follow ttn); it is then classified and handed over
      // first.  The heap operations keep the reference's order (this sift-up, then the next pop's
      // downtree); the next pop's relaxations read ttn and validity only, which sift-ups never touch
      auto early = [&](double key, int cell) {
        if (!AF_INIT_EARLY || finished || h.err || h.ndup || h.ntr < 1 || key < L->hkey[1] ||
            (int)L->hcell[1] == cell)
          return;
        bool f2 = false;
        const int n2 = classify(f2);
        pre_n = n2;
        pre_fin = f2;
        if (n2 > 0) {
          L->njob = n2;
          post(&L->cmd, ++seq);
        }
      };
      if (!pop_two_role(h, seq, jobs, n, posted, early)) h.err = 1;
    }
    post(&L->cmd, -1);
  } else if (tid >= 64) {
    relax_role<LDSMAT>(L, M, c.mv, c.mw, RelaxWin{0, 0, nz - 1, nx - 1, nx, 0, 0, nz, nx, c.dnx, c.dnx, nx, c.quirk},
                       tid - 64);
  }
}

// Decimate the stage grid (every 3rd node) into decT/decC with the hand-over's "outer" test
// (:1719-1753).  All lanes.
AF_DEV void decimate(InitLds* L, int nz, int nx, int lane, int nl) {
  int dz = (nz - 1) / 3 + 1, dx = (nx - 1) / 3 + 1;
  for (int k = lane; k < dz * dx; k += nl) {
    int i = 3 * (k / dx), j = 3 * (k % dx);
    int st = L->S[i * nx + j];
    L->decT[k] = L->T[i * nx + j];
    signed char cls = 0;
    if (st == 0) {
      bool outer = false;
      if (i - 3 >= 0) { if (L->S[(i - 3) * nx + j] == -1) outer = true; } else outer = true;
      if (i + 3 <= nz - 1) { if (L->S[(i + 3) * nx + j] == -1) outer = true; } else outer = true;
      if (j - 3 >= 0) { if (L->S[i * nx + j - 3] == -1) outer = true; } else outer = true;
      if (j + 3 <= nx - 1) { if (L->S[i * nx + j + 3] == -1) outer = true; } else outer = true;
      cls = outer ? 2 : 1;
    } else if (st > 0) {
      cls = 3;
    }
    L->decC[k] = cls;
  }
}

AF_DEV void clear_grid(InitLds* L, int n, int lane, int nl) {
  for (int k = lane; k < n; k += nl) {
    L->T[k] = 0.0;
    L->S[k] = -1;
  }
}


// main loop :2055-2102 on the LDS window (heap in window-local coordinates), two roles as above
template <bool LDSMAT>
AF_DEV void main_prefix(Heap& h, const DevModel& M, const InitJob& J, int wz0, int wx0, int wz1, int wx1,
                        const MidWin& pw, int tid) {
  InitLds* L = h.L;
  const int ww = h.nx;
  const int nnz = M.nz0, nnx = M.nx0;
  const MatView ident{1, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0};
  if (tid < 64) {  // heap role: wavefront 0 (uniform)
    int seq = 0, jobs = 0;
    while (h.ntr > 0 && !h.err) {
      const int lx = h.bx(1), lz = h.bz(1);
      if (L->T[lz * ww + lx] >= J.tstop) break;
      const int iz = lz + wz0, ix = lx + wx0;
      if ((wz0 > 0 && iz - wz0 < 3) || (wz1 < nnz - 1 && wz1 - iz < 3) || (wx0 > 0 && ix - wx0 < 3) ||
          (wx1 < nnx - 1 && wx1 - ix < 3))
        break;
      L->S[lz * ww + lx] = 0;
      int n = 0;
      for (int s = 0; s < 2; s++) {
        const int i = s == 0 ? ix - 1 : ix + 1;
        if (0 <= i && i <= nnx - 1) {
          const int st = L->S[lz * ww + (i - wx0)];
          if (st == -1 || st > 0) {
            L->job[n] = job_pack(lz, i - wx0, st == -1 ? kJobAdd : kJobUpd);
            n++;
          }
        }
      }
      for (int s = 0; s < 2; s++) {
        const int i = s == 0 ? iz - 1 : iz + 1;
        if (0 <= i && i <= nnz - 1) {
          const int st = L->S[(i - wz0) * ww + lx];
          if (st == -1 || st > 0) {
            L->job[n] = job_pack(i - wz0, lx, st == -1 ? kJobAdd : kJobUpd);
            n++;
          }
        }
      }
      if (!pop_two_role(h, seq, jobs, n)) h.err = 1;
    }
    post(&L->cmd, -1);
  } else if (tid >= 64) {
    relax_role<LDSMAT>(L, M, ident, pw, RelaxWin{wz0, wx0, wz1, wx1, ww, wz0, wx0, nnz, nnx, J.dnx, J.dnz, nnz, 0},
                       tid - 64);
  }
}

template <bool LDSMAT>
__global__ __launch_bounds__(128) void fmm_init_kernel(DevModel M0, InitJob* jobs, int njobs, HandoverOut* out) {
  __shared__ InitLds lds;
  InitLds* L = &lds;
  const int src = blockIdx.x;
  crm::lds_init();
  if (src < njobs && threadIdx.x < 16) out[src].prof[threadIdx.x] = 0;
  DevModel M = M0;
  if (LDSMAT) {
    for (int k = threadIdx.x; k < M.nmat; k += blockDim.x) L->mat[k] = M.mtab[k];
    // the small tables the relaxations read: LDS instead of dependent global loads
    if (M.stab && M.nstab <= kInitStab) {
      for (int k = threadIdx.x; k < 5 * M.nstab; k += blockDim.x) L->stab[k] = M.stab[k];
      M.stab = L->stab;
    }
  }
  if (src >= njobs) return;
  const int lane = threadIdx.x, nl = blockDim.x;
#if AF_INIT_DIAG
  if (lane < 12) L->dg[lane] = 0;
#endif
  InitJob J = jobs[src];
  const int nnz = M.nz0, nnx = M.nx0;
  const long isx = J.isx, isz = J.isz;
  HandoverOut* O = out + src;

  const int sgs[3] = {27, 9, 3}, sizes[3] = {2, 6, 13};
  int pisz = 0, pisx = 0, pnz = 0, pnx = 0;
  int err = 0;
  for (int stg = 0; stg < 3; stg++) {
    const int sg = sgs[stg], size = sizes[stg];
    const int left = max(0L, isx - size), right = min((long)nnx - 1, isx + size);
    const int bottom = max(0L, isz - size), top = min((long)nnz - 1, isz + size);
    const int nz = sg * (top - bottom) + 1, nx = sg * (right - left) + 1;
    const int isx_s = sg * (int)(isx - left), isz_s = sg * (int)(isz - bottom);
    StageCfg c;
    c.dnx = J.dnx / sg;
    c.isx = isx_s;
    c.isz = isz_s;
    c.max_dist = sg * size;
    c.quirk = stg == 0;
    c.mv = MatView{sg, (sg - 1) / 2, bottom, sg, (sg - 1) / 2, left, 1, 0, 0, 0, 1};
    c.mw = MidWin{bottom, left, right - left + 1, top - bottom + 1};
    clear_grid(L, nz * nx, lane, nl);
    if (LDSMAT) load_smid(M, L, c.mw, lane, nl);
    __syncthreads();
    Heap h{L, nz, nx, 0, 0};
    if (stg == 0) {
      // straight rays in the source cell footprint (:1546-1590), coarse material at the source
      const int side1 = (sg - 1) / 2;
      MatView ident{1, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0};
      CellMat cs = cell_mat(M, ident, (int)isz, (int)isx);
      const int w = 2 * side1 + 1;
      for (int k = lane; k < w * w; k += nl) {
        int i = k / w - side1, j = k % w - side1;
        if (0 <= isz_s + i && isz_s + i <= nz - 1 && 0 <= isx_s + j && isx_s + j <= nx - 1) {
          double angle = (j == 0) ? 90.0 : AF_ATAN((double)i / (double)j) * kRad2Deg;
          double eff = pymod(cs.veln - angle, 180);
          double velocity = (cs.velpn != 0 || cs.stif == nullptr)
                                ? table_vel(M.gtab, M.ncol, eff, cs.velpn, cs.vm)
                                : christoffel_group(cs.stif, eff, cs.vm);
          double length = c.dnx * sqrt((double)(i * i + j * j));
          L->T[(isz_s + i) * nx + isx_s + j] = length / velocity;
          L->S[(isz_s + i) * nx + isx_s + j] = 0;
        }
      }
      __syncthreads();
      if (lane < 64) {  // (the heap's sift-ups use the whole wavefront 0)
        // window edges -> heap, in the reference's order (:1601-1612)
        const int s1 = side1;
        if (isz_s - s1 >= 0)
          for (int i = max(0, isx_s - s1); i <= min(nx - 1, isx_s + s1); i++) h.add(isz_s - s1, i);
        if (isz_s + s1 <= nz - 1)
          for (int i = max(0, isx_s - s1); i <= min(nx - 1, isx_s + s1); i++) h.add(isz_s + s1, i);
        if (isx_s - s1 >= 0)
          for (int i = max(0, isz_s - s1); i <= min(nz - 1, isz_s + s1); i++) h.add(i, isx_s - s1);
        if (isx_s + s1 <= nx - 1)
          for (int i = max(0, isz_s - s1); i <= min(nz - 1, isz_s + s1); i++) h.add(i, isx_s + s1);
      }
    } else if (lane < 64) {
      // hand-over from the decimated previous stage, in row-major order (:1719-1753)
      int dz = (pnz - 1) / 3 + 1, dx = (pnx - 1) / 3 + 1;
      for (int k = 0; k < dz * dx; k++) {
        int i = 3 * (k / dx), j = 3 * (k % dx);
        int pz = isz_s + (i - pisz) / 3, px = isx_s + (j - pisx) / 3;
        L->T[pz * nx + px] = L->decT[k];
        signed char cls = L->decC[k];
        if (cls == 1 || cls == 2) L->S[pz * nx + px] = 0;
        if (cls >= 2) h.add(pz, px);
      }
    }
    if (lane == 0) {  // control words of the two-role walk
      L->cmd = 0;
      L->done = 0;
    }
    __syncthreads();
    const long long ts = wall_clock64();
    stage_loop<LDSMAT>(h, M, c, lane);
    if (lane == 0) {
      err |= h.err;
      O->prof[stg] = wall_clock64() - ts;
      O->prof[4 + stg] = h.pops;
    }
    __syncthreads();
    if (lane == 0) {
      O->prof[8 + stg] = L->rbusy;
      O->prof[12 + stg] = L->rjobs;
    }
    decimate(L, nz, nx, lane, nl);
    __syncthreads();
    pisz = isz_s;
    pisx = isx_s;
    pnz = nz;
    pnx = nx;
  }
  if (J.exact_r > 0) {
    // ---- exact heap-ordered prefix of the main loop (:2055-2102) in an LDS window ----
    // The reference's pop order (quirky heap included) decides the field near the source, where
    // the wavefront hits grid edges and close hand-over nodes get overwritten.  Run it exactly
    // until the root's T reaches exact_r*dnx/vmax (or the root comes within 3 nodes of a window
    // edge that is not a grid edge), then hand the heap's state to the band kernel.
    const int W = J.exact_r + 6;
    const int wz0 = (int)max(0L, isz - W), wz1 = (int)min((long)nnz - 1, isz + W);
    const int wx0 = (int)max(0L, isx - W), wx1 = (int)min((long)nnx - 1, isx + W);
    const int wh = wz1 - wz0 + 1, ww = wx1 - wx0 + 1;
    if (wh * ww > kInitMaxN) {
      err = 1;
    } else {
      clear_grid(L, wh * ww, lane, nl);
      const MidWin pw = wh * ww <= kInitWin ? MidWin{wz0, wx0, ww, wh} : MidWin{0, 0, 0, 0};
      if (LDSMAT && pw.w) load_smid(M, L, pw, lane, nl);
      __syncthreads();
      Heap h{L, wh, ww, 0, 0};
      if (lane < 64) {
        int dz = (pnz - 1) / 3 + 1, dx = (pnx - 1) / 3 + 1;
        for (int k = 0; k < dz * dx; k++) {
          int i = 3 * (k / dx), j = 3 * (k % dx);
          int pz = (int)(isz + (i - pisz) / 3) - wz0, px = (int)(isx + (j - pisx) / 3) - wx0;
          L->T[pz * ww + px] = L->decT[k];
          signed char cls = L->decC[k];
          if (cls == 1 || cls == 2) L->S[pz * ww + px] = 0;
          if (cls >= 2) h.add(pz, px);
        }
        L->cmd = 0;
        L->done = 0;
      }
      __syncthreads();
      const long long ts = wall_clock64();
      main_prefix<LDSMAT>(h, M, J, wz0, wx0, wz1, wx1, pw, lane);
      if (lane == 0) {
        err |= h.err;
        O->prof[3] = wall_clock64() - ts;
        O->prof[7] = h.pops;
      }
      __syncthreads();
      if (lane == 0) {
        O->prof[11] = L->rbusy;
        O->prof[15] = L->rjobs;
      }
      // emit every touched window node: known (1) / close (3)
      if (lane == 0) {
        int n = 0;
        for (int k = 0; k < wh * ww; k++) {
          int st = L->S[k];
          if (st < 0) continue;
          int z = wz0 + k / ww, x = wx0 + k % ww;
          O->cell[n] = z * nnx + x;
          O->ttn[n] = L->T[k];
          O->cls[n] = st == 0 ? 1 : 3;
          n++;
        }
#if AF_INIT_DIAG
        for (int k = 0; k < 8; k++) O->prof[8 + k] = L->dg[k];
        for (int k = 0; k < 4; k++) O->prof[k] = L->dg[8 + k];  // (diagnostic builds: the stage ticks' slots)
#endif
        O->n = n;
        O->err = err;
      }
      return;
    }
  }
  // emit the decimated stage-3 nodes for the main-grid hand-over (:2006-2040)
  if (lane == 0) {
    int dz = (pnz - 1) / 3 + 1, dx = (pnx - 1) / 3 + 1;
    int n = 0;
    for (int k = 0; k < dz * dx; k++) {
      signed char cls = L->decC[k];
      if (cls == 0) continue;
      int i = 3 * (k / dx), j = 3 * (k % dx);
      long pz = isz + (i - pisz) / 3, px = isx + (j - pisx) / 3;
      O->cell[n] = (int)(pz * nnx + px);
      O->ttn[n] = L->decT[k];
      O->cls[n] = cls;
      n++;
    }
#if AF_INIT_DIAG
    for (int k = 0; k < 8; k++) O->prof[8 + k] = L->dg[k];
    for (int k = 0; k < 4; k++) O->prof[k] = L->dg[8 + k];  // (diagnostic builds: the stage ticks' slots)
#endif
    O->n = n;
    O->err = err;
  }
}

}  // namespace af

extern "C" hipError_t af_launch_init(const af::DevModel* M, af::InitJob* jobs, int njobs, af::HandoverOut* out,
                                     hipStream_t stream) {
  if (M->mid && M->nmat <= af::kInitMat)
    hipLaunchKernelGGL(af::fmm_init_kernel<true>, dim3(njobs), dim3(128), 0, stream, *M, jobs, njobs, out);
  else
    hipLaunchKernelGGL(af::fmm_init_kernel<false>, dim3(njobs), dim3(128), 0, stream, *M, jobs, njobs, out);
  return hipGetLastError();
}
