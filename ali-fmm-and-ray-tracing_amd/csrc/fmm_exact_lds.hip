// fmm_exact_lds.hip — travel_finer_grid()'s exact heap walk (the x9 / x3 stage grids
// Anis_TTF_rays.py:2187-2504 and the fine-grid main loop's prefix :2775-2817) with the walk's
// state in LDS, on gfx950.
//
// fmm_exact.hip keeps the walk's statuses (nsts) in HBM next to the grids, so every pop pays
// memory round trips on its serial path: the neighbours' statuses, the heap index of an updated
// node, the 12-point stencil of a relaxation whose speculative entry went stale, and a store
// drain per relaxation (≈7.7 µs per pop on the weld example, 50 % of the wave's cycles waiting,
// profiles/r4exact_*).  Here only the travel times stay in HBM; everything the walk decides on
// is in LDS:
//   * statuses as 2-bit codes (far / close / known) of every node of the current grid (stage
//     grids whole, up to 163 840 nodes = subgrid 9; the fine main grid as a window around the
//     source that covers the prefix);
//   * the heap (keys = copies of ttn, as in fmm_exact.hip) with, per entry, the node and the slot
//     of the node's heap index in an LDS hash (node -> the reference's nsts > 0), so sifts write
//     heap indices without a lookup;
//   * per lane, a speculative relaxation (node, value, update()'s stencil stage, material) whose
//     12-point stencil is kept current in LDS: every committed relaxation patches the stencils
//     that contain its node, so a stale entry is re-checked (stencil stage re-run, finish only if
//     it changed) without any memory access.  Only relaxations with no entry cost a memory round
//     trip: one evaluation pass in which lane 0 evaluates the job and the other lanes guesses (the
//     neighbours of the heap's first 16 entries), as in fmm_exact.hip.
// The walk, its heap (round-half-even parent, SURVEY B-D3), duplicate entries (the stage-1 window
// corners, :2277-2288) and the hand-over order are fmm_exact.hip's, which reproduces the
// reference's; results are bit-identical to it (tests/test_gpu_parity.py weld sg 3 / 9 fields,
// tools/weld_split.py --dump).  Larger grids (subgrid > 9) and heap overflows use fmm_exact.hip.
#define CR_LDS_TABLES  // cr_math.h tables in LDS (crm::lds_init at kernel start)
#include "kernels.h"
#include "local_ops.h"
#include "fields.h"

namespace af {
namespace xl {

constexpr int kThreads = 256;  // 4 waves clear and hand over; wave 0 walks
#ifndef AF_XL_DIAG
#define AF_XL_DIAG 0  // diagnostic build: cycle counters of the walk (walk(), BandSrc::ph / sub)
#endif
// a stale speculative entry's stencil stage re-run across the wavefront (1) or on its lane (0)
#ifndef AF_XL_PARSEL
#define AF_XL_PARSEL 1
#endif
#ifndef AF_XL_TWO_ROLE
#define AF_XL_TWO_ROLE 1  // heap wavefront + relax wavefront (1), or one wavefront doing both (0)
#endif
constexpr int kCap = 163840;   // status nodes (2 bits each): stage grids up to 404 x 404
constexpr int kHeap = 4096;    // heap slots (1-based)
constexpr int kHTLog = 13;
constexpr int kHT = 1 << kHTLog;  // hash slots (node -> heap index)
constexpr int kDec = 18432;       // decimated nodes of a stage grid (hand-over classes)
constexpr int kDup = 8;           // nodes with two heap entries

constexpr unsigned kLive = 1u << 30, kTomb = 0x80000000u;  // hash words: live | pos << 18 | node
constexpr unsigned kNodeM = (1u << 18) - 1;
constexpr unsigned kDupF = 0x80000000u;  // heap entry: node | hash slot << 18 | kDupF
constexpr unsigned kSFar = 0, kSClose = 1, kSKnown = 2;

struct Lds {
  unsigned st[kCap / 16];
  double key[kHeap];
  unsigned ent[kHeap];
  unsigned ht[kHT];
  double stn[12][64];  // per-lane speculative stencils, [stencil slot][lane]
  signed char dec[kDec];
  int dup[kDup];
  int nused;  // hash slots that are live or tombstones
  // two-role walk (heap wavefront -> relax wavefront): command sequence number (-1 stop), the
  // pop's relaxation jobs (node | fresh << 31), relaxations done / applied to the heap (running
  // counts), their values, the heap size (for the relax role's guesses), serial (see heap_role)
  int cmd, done, applied, njob, serial, ntr_hint;
  int job[4];
  double jval[4];
};

AF_DEV double rlane(double v, int l) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

AF_DEV unsigned sget(const Lds* L, int c) { return (L->st[c >> 4] >> ((c & 15) * 2)) & 3u; }
AF_DEV void sset(Lds* L, int c, unsigned v) {  // any previous state (LDS atomics: lanes share words)
  const unsigned sh = (c & 15) * 2;
  atomicAnd(&L->st[c >> 4], ~(3u << sh));
  if (v) atomicOr(&L->st[c >> 4], v << sh);
}

AF_DEV unsigned hslot(int c) { return ((unsigned)c * 2654435761u) >> (32 - kHTLog); }

// the grid of a walk: T in HBM (row-major nz x nx, far = NaN), statuses of the window rows
// [wz0, wz0 + wh), columns [wx0, wx0 + ww) in LDS (stage grids: the whole grid)
struct XG {
  double* T;
  int nz, nx;
  int wz0, wx0, wh, ww;
  MatView mv;
  double dnx, dnz;
  AF_DEV bool inw(int z, int x) const { return z >= wz0 && z < wz0 + wh && x >= wx0 && x < wx0 + ww; }
  AF_DEV int loc(int z, int x) const { return (z - wz0) * ww + (x - wx0); }
  AF_DEV int gz(int c) const { return wz0 + c / ww; }
  AF_DEV int gx(int c) const { return wx0 + c % ww; }
};

// status accessor for fouds18_A() (known = 0, close = 1, far = -1) with T from HBM (far -> 0)
struct XField {
  const Lds* L;
  const XG* g;
  AF_DEV int st(long z, long x) const {
    if (z >= g->nz || !g->inw((int)z, (int)x)) return -1;
    const unsigned s = sget(L, g->loc((int)z, (int)x));
    return s == kSKnown ? 0 : s == kSClose ? 1 : -1;
  }
  AF_DEV double tt(long z, long x) const {
    if (z >= g->nz || z < 0 || x < 0 || x >= g->nx) return 0.0;
    return far0(gld(g->T + z * g->nx + x));
  }
};

// addtree / updtree / downtree (:94-237) with the heap indices (nsts > 0) in the LDS hash.  A heap
// index write (setpos) is one LDS store through the entry's hash slot; an entry of a node with two
// heap entries (kDupF) also makes the node close again, as the reference's nsts = index does after
// the node was popped through its other entry.  Lane 0 only.
struct Heap {
  Lds* L;
  int ntr = 0, err = 0, ndup = 0;
  int livedup = 0;  // heap entries carrying kDupF
  AF_DEV static int parent(int t) {  // round(t / 2), half-even (:123)
    const int m = t >> 1;
    return (t & 1) ? ((m & 1) ? m + 1 : m) : m;
  }
  AF_DEV bool isdup(int c) const {
    bool d = false;
    for (int k = 0; k < ndup; k++) d |= L->dup[k] == c;
    return d;
  }
  AF_DEV int hfind(int c) const {
    unsigned s = hslot(c);
    for (int p = 0; p < kHT; p++) {
      const unsigned w = L->ht[s];
      if (w == 0u) return -1;
      if ((w >> 30) == 1u && (int)(w & kNodeM) == c) return (int)s;
      s = (s + 1) & (kHT - 1);
    }
    return -1;
  }
  AF_DEV int hinsert(int c) {
    unsigned s = hslot(c);
    while (true) {
      const unsigned w = L->ht[s];
      if (w == 0u || w == kTomb) {
        if (w == 0u) L->nused++;
        L->ht[s] = kLive | (unsigned)c;
        return (int)s;
      }
      s = (s + 1) & (kHT - 1);
    }
  }
  AF_DEV int pos_of(int c) const { return (int)((L->ht[hfind(c)] >> 18) & 0xfffu); }
  AF_DEV void setpos(unsigned e, int pos) {
    L->ht[(e >> 18) & (kHT - 1)] = kLive | ((unsigned)pos << 18) | (e & kNodeM);
    if (e & kDupF) sset(L, (int)(e & kNodeM), kSClose);
  }
  AF_DEV void sift_up(int tpc, double km) {
    const unsigned em = L->ent[tpc];
    int tpp = parent(tpc);
    while (tpp > 0) {
      const double kp = L->key[tpp];
      unsigned ep = L->ent[tpp];
      asm volatile("" : "+v"(ep));  // both reads in one LDS round trip (not the entry after the compare)
      if (!(km < kp)) break;
      setpos(em, tpp);
      setpos(ep, tpc);
      L->ent[tpc] = ep;
      L->key[tpc] = kp;
      tpc = tpp;
      tpp = parent(tpc);
    }
    L->ent[tpc] = em;
    L->key[tpc] = km;
  }
  // key = the node's ttn; fresh: the node is far (a relaxation of a far neighbour)
  AF_DEV void add(int c, double key, bool fresh) {
    ntr += 1;
    if (ntr >= kHeap) {
      err = 9;
      ntr = kHeap - 1;
      return;
    }
    const unsigned s0 = fresh ? kSFar : sget(L, c);
    unsigned e;
    if (s0 == kSClose) {  // already in the heap: a second entry
      if (ndup == kDup) {
        err = 9;
        return;
      }
      L->dup[ndup++] = c;
      const int hs = hfind(c);
      for (int k = 1; k < ntr; k++)  // its other entries now carry the flag
        if ((int)(L->ent[k] & kNodeM) == c && !(L->ent[k] & kDupF)) {
          L->ent[k] |= kDupF;
          livedup++;
        }
      e = (unsigned)c | ((unsigned)hs << 18) | kDupF;
    } else {
      int hs = fresh ? -1 : hfind(c);  // a popped node with two entries keeps its slot
      if (hs < 0) hs = hinsert(c);
      e = (unsigned)c | ((unsigned)hs << 18) | (!fresh && isdup(c) ? kDupF : 0u);
      sset(L, c, kSClose);
    }
    if (e & kDupF) livedup++;
    L->ent[ntr] = e;
    setpos(e, ntr);
    sift_up(ntr, key);
  }
  // returns whether the node has another heap entry (its keys then follow, sync)
  AF_DEV bool upd(int c, double key) {
    const int tpc = pos_of(c);
    L->key[tpc] = key;
    const bool d = (L->ent[tpc] & kDupF) != 0u;
    sift_up(tpc, key);
    return d;
  }
  // node c (with two heap entries) has ttn key now: every entry of it takes it
  AF_DEV void sync(int c, double key) {
    for (int k = 1; k <= ntr; k++)
      if ((int)(L->ent[k] & kNodeM) == c) L->key[k] = key;
  }
  // pop the root (its status -> known, its heap-index slot freed unless the node has another
  // entry), then downtree
  AF_DEV void pop() {
    pop_known();
    pop_rest();
  }
  AF_DEV void pop_known() { sset(L, (int)(L->ent[1] & kNodeM), kSKnown); }
  AF_DEV void pop_rest() {
    const unsigned e0 = L->ent[1];
    if (!(e0 & kDupF)) L->ht[(e0 >> 18) & (kHT - 1)] = kTomb;
    else livedup--;
    if (ntr == 1) {
      ntr = 0;
      return;
    }
    const unsigned em = L->ent[ntr];
    const double km = L->key[ntr];
    setpos(em, 1);
    ntr -= 1;
    int tpp = 1, tpc = 2;
    while (tpc < ntr) {
      const double k1 = L->key[tpc], k2 = L->key[tpc + 1];
      unsigned e1 = L->ent[tpc], e2 = L->ent[tpc + 1];
      asm volatile("" : "+v"(e1), "+v"(e2));  // keys and entries in one LDS round trip
      const bool right = k1 > k2;
      const int t = right ? tpc + 1 : tpc;
      const double kc = right ? k2 : k1;
      const unsigned ec = right ? e2 : e1;
      if (kc < km) {
        setpos(em, t);
        setpos(ec, tpp);
        L->ent[tpp] = ec;
        L->key[tpp] = kc;
        tpp = t;
        tpc = 2 * tpp;
      } else {
        tpc = ntr + 1;
      }
    }
    if (tpc == ntr) {
      const double kc = L->key[tpc];
      const unsigned ec = L->ent[tpc];
      if (kc < km) {
        setpos(em, tpc);
        setpos(ec, tpp);
        L->ent[tpp] = ec;
        L->key[tpp] = kc;
        tpp = tpc;
      }
    }
    L->ent[tpp] = em;
    L->key[tpp] = km;
  }
};

// Rebuild the hash without its tombstones (wave 0, every lane): each heap entry's node is
// re-inserted with the heap index of that entry (nodes with two entries: the index the old slot
// held) and the entry takes the new slot.
AF_DEV void rehash(Lds* L, Heap& h, int lane) {
  int ntr = __shfl(h.ntr, 0), nd = __shfl(h.ndup, 0);
  // the heap indices of the nodes with two entries, before the table is cleared
  int dpos = -1, dnode = -1;
  if (lane < nd) {
    dnode = L->dup[lane];
    unsigned s = hslot(dnode);
    for (int p = 0; p < kHT; p++) {
      const unsigned w = L->ht[s];
      if (w == 0u) break;
      if ((w >> 30) == 1u && (int)(w & kNodeM) == dnode) {
        dpos = (int)((w >> 18) & 0xfffu);
        break;
      }
      s = (s + 1) & (kHT - 1);
    }
  }
  for (int k = lane; k < kHT; k += 64) L->ht[k] = 0u;
  for (int k = 1 + lane; k <= ntr; k += 64) {
    const unsigned e = L->ent[k];
    const int c = (int)(e & kNodeM);
    unsigned s = hslot(c);
    while (true) {
      const unsigned prev = atomicCAS(&L->ht[s], 0u, kLive | ((unsigned)k << 18) | (unsigned)c);
      if (prev == 0u || (int)(prev & kNodeM) == c) break;
      s = (s + 1) & (kHT - 1);
    }
    L->ent[k] = (e & ~(((unsigned)(kHT - 1)) << 18)) | (s << 18);
  }
  // popped nodes with two entries keep a slot even with no entry left
  if (lane < nd && dpos >= 0) {
    unsigned s = hslot(dnode);
    while (true) {
      const unsigned prev = atomicCAS(&L->ht[s], 0u, kLive | ((unsigned)dpos << 18) | (unsigned)dnode);
      if (prev == 0u) break;
      if ((int)(prev & kNodeM) == dnode) {
        L->ht[s] = kLive | ((unsigned)dpos << 18) | (unsigned)dnode;
        break;
      }
      s = (s + 1) & (kHT - 1);
    }
  }
  int used = 0;
  for (int k = lane; k < kHT; k += 64) used += L->ht[k] != 0u;
  for (int o = 32; o > 0; o >>= 1) used += __shfl_xor(used, o);
  if (lane == 0) L->nused = used;
}

// One lane's speculative relaxation: node (window-local, -1: none), grid coordinates, value,
// update()'s stencil stage and the node's material; its stencil values live in Lds::stn.
struct Spec {
  int c, z, x;
  unsigned vm;
  bool dirty;
  double v;
  UpdSel sel;
  CellMat cm;
};

// every lane: committed relaxation (rz, rx) = v -> the stencils that contain it
AF_DEV void patch(Lds* L, Spec& sp, int rz, int rx, double v, int lane) {
  if (sp.c < 0) return;
  const int dz = rz - sp.z, dx = rx - sp.x;
  const int ad = abs(dz) + abs(dx);
  if (ad == 0 || ad > 2 || (dz != 0 && dx != 0 && (abs(dz) != 1 || abs(dx) != 1))) return;
  const int k = NbField::slot(dz, dx);
  L->stn[k][lane] = v;
  sp.vm |= 1u << k;
  sp.dirty = true;
}

AF_DEV void stencil_from_lds(const Lds* L, const Spec& sp, NbFieldT& nb, int lane) {
  nb.iz = sp.z;
  nb.ix = sp.x;
  nb.vm = sp.vm;
  nb.t0 = L->stn[0][lane]; nb.t1 = L->stn[1][lane]; nb.t2 = L->stn[2][lane]; nb.t3 = L->stn[3][lane];
  nb.t4 = L->stn[4][lane]; nb.t5 = L->stn[5][lane]; nb.t6 = L->stn[6][lane]; nb.t7 = L->stn[7][lane];
  nb.t8 = L->stn[8][lane]; nb.t9 = L->stn[9][lane]; nb.t10 = L->stn[10][lane]; nb.t11 = L->stn[11][lane];
}

// update() of the job (rz, rx) on the current state (wave 0, every lane; wave-uniform result).
// An entry for the node: its stencil is current (patched), so its value stands if the stencil
// stage is unchanged, else the finish runs on the entry's lane.  No entry: one evaluation pass —
// the job on lane 0, and on every other lane a guess (a neighbour of one of the heap's first 16
// entries that is not known), each loading its stencil and material from memory.
AF_DEV double relax_value(Lds* L, const DevModel& M, const XG& g, Spec& sp, int r, int rz, int rx, int ntr,
                          int lane, long long& npass, int& path) {
  const unsigned long long hm = __ballot(sp.c == r);
  if (hm) {
    const int e = __ffsll((long long)hm) - 1;
    int pth = 0;
    if (__builtin_amdgcn_readlane((int)sp.dirty, e)) {
      // the patched stencil's stage again, spread over the wavefront (lane k < 12: slot k of the
      // entry's stencil; lanes 0..7 a square stencil each), on the entry's lane where update()
      // runs its triangular stage
      const unsigned vm_e = (unsigned)__builtin_amdgcn_readlane((int)sp.vm, e);
      const int z_e = __builtin_amdgcn_readlane(sp.z, e), x_e = __builtin_amdgcn_readlane(sp.x, e);
      const double tk = lane < 12 ? L->stn[lane][e] : 0.0;
      const bool vk = lane < 12 && ((vm_e >> lane) & 1u);
      UpdSel s2;
      const bool par = AF_XL_PARSEL && update_select_lanes(tk, vk, z_e, x_e, g.nz, g.nx, lane, s2);
      if (lane == e) {
        if (!par) {
          NbFieldT nb;
          stencil_from_lds(L, sp, nb, lane);
          s2 = update_nb_select(nb, sp.z, sp.x, g.nz, g.nx);
        }
        pth = 1;
        if (!s2.same(sp.sel)) {
          sp.v = update_nb_finish_ool(M, sp.cm, sp.z, sp.x, g.dnx, s2);
          sp.sel = s2;
          pth = 2;
        }
        sp.dirty = false;
      }
    }
    path = __builtin_amdgcn_readlane(pth, e);
    return rlane(sp.v, e);
  }
  path = 3;
  npass++;
  int cz = rz, cx = rx;
  bool cand = true;
  if (lane > 0) {
    const int p = 1 + ((lane - 1) >> 2), d = (lane - 1) & 3;
    const int hc = (int)(L->ent[p] & kNodeM);
    cz = g.gz(hc) + (d == 2 ? -1 : d == 3 ? 1 : 0);
    cx = g.gx(hc) + (d == 0 ? -1 : d == 1 ? 1 : 0);
    cand = p <= ntr && cz >= 0 && cz < g.nz && cx >= 0 && cx < g.nx && g.inw(cz, cx) &&
           sget(L, g.loc(cz, cx)) != kSKnown;
  }
  if (cand) {
    sp.cm = cell_mat(M, g.mv, cz, cx);
    NbFieldT nb;
    nb.load(g.T, g.nz, g.nx, cz, cx);
    L->stn[0][lane] = nb.t0; L->stn[1][lane] = nb.t1; L->stn[2][lane] = nb.t2; L->stn[3][lane] = nb.t3;
    L->stn[4][lane] = nb.t4; L->stn[5][lane] = nb.t5; L->stn[6][lane] = nb.t6; L->stn[7][lane] = nb.t7;
    L->stn[8][lane] = nb.t8; L->stn[9][lane] = nb.t9; L->stn[10][lane] = nb.t10; L->stn[11][lane] = nb.t11;
    sp.vm = nb.vm;
    sp.sel = update_nb_select(nb, cz, cx, g.nz, g.nx);
    sp.v = update_nb_finish_ool(M, sp.cm, cz, cx, g.dnx, sp.sel);
    sp.c = g.loc(cz, cx);
    sp.z = cz;
    sp.x = cx;
    sp.dirty = false;
  } else {
    sp.c = -1;
  }
  return rlane(sp.v, 0);
}

// The heap walk (:2292-2346, :2460-2504, :2775-2817) on wave 0.  stage: stop when a popped node's
// neighbour falls off the stage grid at max_dist + 1 from the source; main grid: stop when the
// root reaches tstop or comes within 3 nodes of a window edge that is not a grid edge.  Returns
// the pops.
AF_DEV long long walk(Lds* L, Heap& h, const DevModel& M, const XG& g, bool stage, int isx_s, int isz_s,
                      int max_dist, double tstop, Spec& sp, int lane, long long* prof, long long* dgo) {
  long long pops = 0, nrel = 0, npass = 0;
  // diagnostic build (AF_XL_DIAG): shader-clock cycles of pop, relaxation value by path (clean
  // entry / stencil stage unchanged / finish / evaluation pass), commit, and the path counts
  long long dg[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  bool finished = false;
  while (true) {
    int go = 0, c = 0, ntr = 0;
    if (lane == 0) {
      if (L->nused > (kHT * 3) / 4) go = -1;  // rehash first
      else go = h.ntr > 0 && !finished && !h.err && !(tstop > 0 && L->key[1] >= tstop);
      c = (int)(L->ent[1] & kNodeM);
      ntr = h.ntr;
    }
    go = __shfl(go, 0);
    if (go < 0) {
      rehash(L, h, lane);
      continue;
    }
    if (!go) break;
    c = __shfl(c, 0);
    ntr = __shfl(ntr, 0);
    const int iz = g.gz(c), ix = g.gx(c);
    if (!stage && ((g.wz0 > 0 && iz - g.wz0 < 3) || (g.wz0 + g.wh < g.nz && g.wz0 + g.wh - 1 - iz < 3) ||
                   (g.wx0 > 0 && ix - g.wx0 < 3) || (g.wx0 + g.ww < g.nx && g.wx0 + g.ww - 1 - ix < 3))) {
      // the window edge before tstop (the root key is still below it): the HBM walk redoes the
      // source (error 9), so the hand-over is the reference's prefix to tstop
      if (lane == 0) h.err = 9;
      break;
    }  // the window holds no more of the prefix (the band kernel goes on from the heap)
    // lanes 0..3: neighbour x-1, x+1, z-1, z+1; statuses read before downtree (fmm_exact.hip)
    const int kz = lane == 2 ? iz - 1 : lane == 3 ? iz + 1 : iz;
    const int kx = lane == 0 ? ix - 1 : lane == 1 ? ix + 1 : ix;
    const bool inb = lane < 4 && (lane < 2 ? (0 <= kx && kx <= g.nx - 1) : (0 <= kz && kz <= g.nz - 1));
    const unsigned st = inb ? sget(L, g.loc(kz, kx)) : kSKnown;
    const bool edge = lane < 4 && !inb && stage && (lane < 2 ? abs(isx_s - kx) : abs(isz_s - kz)) == max_dist + 1;
    const unsigned long long jm = __ballot(inb && st != kSKnown);
    if (__ballot(edge) != 0ull) finished = true;
    const unsigned long long fm = __ballot(inb && st == kSFar);
    const long long tp0 = AF_XL_DIAG ? clock64() : 0;
    if (lane == 0) h.pop();
    if (AF_XL_DIAG) dg[0] += clock64() - tp0;
    pops++;
    for (int k = 0; k < 4; k++) {
      if (!((jm >> k) & 1ull)) continue;
      const int rz = k == 2 ? iz - 1 : k == 3 ? iz + 1 : iz, rx = k == 0 ? ix - 1 : k == 1 ? ix + 1 : ix;
      const int r = g.loc(rz, rx);
      const long long td0 = AF_XL_DIAG ? clock64() : 0;
      int path = 0;
      double v = relax_value(L, M, g, sp, r, rz, rx, ntr, lane, npass, path);
      const long long td1 = AF_XL_DIAG ? clock64() : 0;
      if (AF_XL_DIAG) dg[1 + path] += td1 - td0;
      if (AF_XL_DIAG && path == 1) dg[7]++;
      if (AF_XL_DIAG && path == 2) dg[8]++;
      nrel++;
      if (lane == 0) {
        if (v == -1.0) {
          const XField F{L, &g};
          v = fouds18(F, M, cell_mat(M, g.mv, rz, rx), rz, rx, g.dnx, g.dnz, g.nx, g.nz, mat_slo(M, g.mv, rz, rx));
        }
        gst(g.T + (long)rz * g.nx + rx, v);
        // a far node's new entry is its only one; an updated node's entry says whether it has two
        if ((fm >> k) & 1ull) h.add(r, v, true);
        else if (h.upd(r, v)) h.sync(r, v);
      }
      v = rlane(v, 0);
      patch(L, sp, rz, rx, v, lane);
      ntr = __shfl(h.ntr, 0);
      if (AF_XL_DIAG) dg[5] += clock64() - td1;
    }
  }
  if (prof && lane == 0) {  // diagnostics: relaxations, evaluation passes (BandSrc::sub)
    prof[0] += nrel;
    prof[1] += npass;
    if (AF_XL_DIAG) {  // BandSrc::ph[0..5] and sub[2..3] (the band kernel writes them only when profiling)
      for (int k = 0; k < 6; k++) dgo[k] += dg[k];
      prof[2] += dg[7];
      prof[3] += dg[8];
    }
  }
  return pops;
}

// ---- the walk over two wavefronts (AF_XL_TWO_ROLE) ----
// The heap wavefront pops, classifies the popped node's neighbours (far -> addtree, close ->
// updtree, read before downtree as in walk()), makes the node known and hands the relaxation jobs
// to the relax wavefront, then runs downtree while the relaxations are evaluated, and each job's
// addtree / updtree as soon as its value is posted.  The relax wavefront evaluates the jobs in
// order (speculative entries / evaluation passes / fouds18_A(), walk()'s relax_value) and stores
// T.  update() reads T and validity only, which neither downtree nor addtree / updtree change, so
// the values are walk()'s.  fouds18_A() reads known-ness, which the heap side changes only through
// a node with two heap entries (setpos makes it close again): while such entries are in the heap
// (Heap::livedup) the heap runs downtree before posting the jobs and the relax side waits for the
// earlier jobs' addtree / updtree before a fouds18_A() — the sequential order.
AF_DEV void xpost(int* w, int v) { __hip_atomic_store(w, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); }
AF_DEV int xload(int* w) { return __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); }
// polls back off with s_sleep(AF_XL_SLEEP) (0: spin)
#ifndef AF_XL_SLEEP
#define AF_XL_SLEEP 1
#endif
AF_DEV bool xawait_at_least(int* w, int v) {  // false: timeout (the other role is gone)
  for (long spins = 0; xload(w) < v; spins++) {
    if (AF_XL_SLEEP) __builtin_amdgcn_s_sleep(AF_XL_SLEEP);
    if (spins > (1L << 28)) return false;
  }
  return true;
}
AF_DEV int xawait_change(int* w, int last) {  // the next value != last, or -2 on timeout
  for (long spins = 0;; spins++) {
    const int v = xload(w);
    if (v != last) return v;
    if (AF_XL_SLEEP) __builtin_amdgcn_s_sleep(AF_XL_SLEEP);
    if (spins > (1L << 28)) return -2;
  }
}

// heap wavefront (every lane; lane 0 holds the heap).  Returns the pops.
AF_DEV long long heap_role(Lds* L, Heap& h, const XG& g, bool stage, int isx_s, int isz_s, int max_dist,
                           double tstop, int lane, long long* dgo) {
  long long pops = 0;
  long long dg[4] = {0, 0, 0, 0};  // AF_XL_DIAG: waits for relaxations, downtree, addtree / updtree, the rest
  long long tl = AF_XL_DIAG ? clock64() : 0;
  bool finished = false;
  int seq = 0, jobs = 0;
  while (true) {
    int go = 0, c = 0;
    if (lane == 0) {
      if (L->nused > (kHT * 3) / 4) go = -1;  // rehash first
      else go = h.ntr > 0 && !finished && !h.err && !(tstop > 0 && L->key[1] >= tstop);
      c = (int)(L->ent[1] & kNodeM);
    }
    go = __shfl(go, 0);
    if (go < 0) {
      rehash(L, h, lane);
      continue;
    }
    if (!go) break;
    c = __shfl(c, 0);
    const int iz = g.gz(c), ix = g.gx(c);
    if (!stage && ((g.wz0 > 0 && iz - g.wz0 < 3) || (g.wz0 + g.wh < g.nz && g.wz0 + g.wh - 1 - iz < 3) ||
                   (g.wx0 > 0 && ix - g.wx0 < 3) || (g.wx0 + g.ww < g.nx && g.wx0 + g.ww - 1 - ix < 3))) {
      // the window edge before tstop (the root key is still below it): the HBM walk redoes the
      // source (error 9), so the hand-over is the reference's prefix to tstop
      if (lane == 0) h.err = 9;
      break;
    }
    const int kz = lane == 2 ? iz - 1 : lane == 3 ? iz + 1 : iz;
    const int kx = lane == 0 ? ix - 1 : lane == 1 ? ix + 1 : ix;
    const bool inb = lane < 4 && (lane < 2 ? (0 <= kx && kx <= g.nx - 1) : (0 <= kz && kz <= g.nz - 1));
    const unsigned st = inb ? sget(L, g.loc(kz, kx)) : kSKnown;
    const bool edge = lane < 4 && !inb && stage && (lane < 2 ? abs(isx_s - kx) : abs(isz_s - kz)) == max_dist + 1;
    const unsigned long long jm = __ballot(inb && st != kSKnown);
    if (__ballot(edge) != 0ull) finished = true;
    const unsigned long long fm = __ballot(inb && st == kSFar);
    const int n = __popcll(jm);
    pops++;
    if (lane == 0) {
      h.pop_known();  // the popped node is known before any relaxation of this pop (fouds18_A)
      const bool serial = h.livedup > 0;
      if (serial || n == 0) h.pop_rest();
      if (n > 0) {
        int q = 0;
        for (int k = 0; k < 4; k++) {
          if (!((jm >> k) & 1ull)) continue;
          const int rz = k == 2 ? iz - 1 : k == 3 ? iz + 1 : iz, rx = k == 0 ? ix - 1 : k == 1 ? ix + 1 : ix;
          L->job[q++] = g.loc(rz, rx) | (((fm >> k) & 1ull) ? (int)0x80000000 : 0);
        }
        L->njob = n;
        L->serial = serial ? 1 : 0;
        L->ntr_hint = h.ntr;
        xpost(&L->cmd, ++seq);
        long long t1 = AF_XL_DIAG ? clock64() : 0;
        if (AF_XL_DIAG) dg[3] += t1 - tl;
        if (!serial) h.pop_rest();  // downtree beside the relaxations
        if (AF_XL_DIAG) {
          const long long t2 = clock64();
          dg[1] += t2 - t1;
          t1 = t2;
        }
        for (int q2 = 0; q2 < n; q2++) {
          if (!xawait_at_least(&L->done, jobs + q2 + 1)) {
            h.err = 10;
            break;
          }
          long long t3 = AF_XL_DIAG ? clock64() : 0;
          if (AF_XL_DIAG) dg[0] += t3 - t1;
          const int jw = L->job[q2];
          const int r = jw & 0x7fffffff;
          const double v = L->jval[q2];
          if (jw < 0) h.add(r, v, true);
          else if (h.upd(r, v)) h.sync(r, v);
          xpost(&L->applied, jobs + q2 + 1);
          if (AF_XL_DIAG) {
            t1 = clock64();
            dg[2] += t1 - t3;
          }
        }
        if (AF_XL_DIAG) tl = t1;
        jobs += n;
      }
    }
  }
  if (lane == 0) xpost(&L->cmd, -1);
  if (AF_XL_DIAG && lane == 0)
    for (int k = 0; k < 4; k++) dgo[k] += dg[k];
  return pops;
}

// relax wavefront (every lane)
AF_DEV void relax_role(Lds* L, const DevModel& M, const XG& g, Spec& sp, int lane, long long* prof,
                       long long* dgo) {
  long long nrel = 0, npass = 0;
  long long dg[2] = {0, 0};  // AF_XL_DIAG: waits for a command, the rest
  int last = 0, jobs = 0;
  sp.c = -1;
  while (true) {
    int cmd = 0;
    const long long tw = AF_XL_DIAG ? clock64() : 0;
    if (lane == 0) cmd = xawait_change(&L->cmd, last);
    cmd = __shfl(cmd, 0);
    const long long tw2 = AF_XL_DIAG ? clock64() : 0;
    if (AF_XL_DIAG) dg[0] += tw2 - tw;
    if (cmd < 0) break;  // stop (or timeout: the heap wavefront is gone)
    last = cmd;
    const int n = L->njob, serial = L->serial, ntr = L->ntr_hint;
    const int4 jv = *reinterpret_cast<const int4*>(L->job);
    for (int q = 0; q < n; q++) {
      const int jw = q == 0 ? jv.x : q == 1 ? jv.y : q == 2 ? jv.z : jv.w;
      const int r = jw & 0x7fffffff;
      const int rz = g.gz(r), rx = g.gx(r);
      int path = 0;
      double v = relax_value(L, M, g, sp, r, rz, rx, ntr, lane, npass, path);
      nrel++;
      if (lane == 0) {
        if (v == -1.0) {
          if (serial) xawait_at_least(&L->applied, jobs + q);  // the earlier jobs' heap updates first
          const XField F{L, &g};
          v = fouds18(F, M, cell_mat(M, g.mv, rz, rx), rz, rx, g.dnx, g.dnz, g.nx, g.nz, mat_slo(M, g.mv, rz, rx));
        }
        gst(g.T + (long)rz * g.nx + rx, v);
        L->jval[q] = v;
        xpost(&L->done, jobs + q + 1);
      }
      v = rlane(v, 0);
      patch(L, sp, rz, rx, v, lane);
    }
    jobs += n;
    if (AF_XL_DIAG) dg[1] += clock64() - tw2;
  }
  if (prof && lane == 0) {
    prof[0] += nrel;
    prof[1] += npass;
  }
  if (AF_XL_DIAG && lane == 0) {
    dgo[4] += dg[0];
    dgo[5] += dg[1];
  }
}

// all threads: the hand-over class of every 3rd node of the grid just walked (:2391-2425,
// :2725-2759): 0 far, 1 known, 2 known with a far (or missing) node 3 away = "outer", 3 close
AF_DEV void classify(Lds* L, int nz, int nx, int tid) {
  const int dz = (nz - 1) / 3 + 1, dx = (nx - 1) / 3 + 1;
  for (int k = tid; k < dz * dx; k += kThreads) {
    const int i = 3 * (k / dx), j = 3 * (k % dx);
    const unsigned s = sget(L, i * nx + j);
    signed char cls = 0;
    if (s == kSKnown) {
      bool outer = false;
      if (i - 3 >= 0) { if (sget(L, (i - 3) * nx + j) == kSFar) outer = true; } else outer = true;
      if (i + 3 <= nz - 1) { if (sget(L, (i + 3) * nx + j) == kSFar) outer = true; } else outer = true;
      if (j - 3 >= 0) { if (sget(L, i * nx + j - 3) == kSFar) outer = true; } else outer = true;
      if (j + 3 <= nx - 1) { if (sget(L, i * nx + j + 3) == kSFar) outer = true; } else outer = true;
      cls = outer ? 2 : 1;
    } else if (s == kSClose) {
      cls = 3;
    }
    L->dec[k] = cls;
  }
}

AF_DEV void clear_state(Lds* L, int nst, int tid) {
  for (int k = tid; k < (nst + 15) / 16; k += kThreads) L->st[k] = 0u;
  for (int k = tid; k < kHT; k += kThreads) L->ht[k] = 0u;
  if (tid == 0) L->nused = 0;
}

AF_DEV void clear_grid(double* T, long n, int tid) {
  const double nan = __builtin_nan("");
  for (long k = tid; k < n; k += kThreads) gst(T + k, nan);
}

// wave 0: the hand-over from the previous grid s (classes in Lds::dec, T in HBM) into g, in
// row-major order: T copied, known nodes known, outer-known and close nodes into the heap (add,
// not fresh).  Chunks of 64 nodes: one memory round trip for the chunk's T, then lane 0 adds its
// heap nodes in order.
AF_DEV void handover(Lds* L, Heap& h, const double* sT, int snz, int snx, int isz_s, int isx_s, const XG& g, int isz_d,
                     int isx_d, int lane) {
  const int dz = (snz - 1) / 3 + 1, dx = (snx - 1) / 3 + 1, n = dz * dx;
  for (int k0 = 0; k0 < n; k0 += 64) {
    const int k = k0 + lane;
    int cls = 0, c = 0;
    double t = 0.0;
    if (k < n) {
      const int i = 3 * (k / dx), j = 3 * (k % dx);
      const int pz = isz_d + (i - isz_s) / 3, px = isx_d + (j - isx_s) / 3;
      cls = L->dec[k];
      t = gld(sT + (long)i * snx + j);
      gst(g.T + (long)pz * g.nx + px, t);
      c = g.loc(pz, px);
      if (cls == 1 || cls == 2) sset(L, c, kSKnown);
    }
    unsigned long long am = __ballot(k < n && cls >= 2);
    while (am) {
      const int l = __ffsll((long long)am) - 1;
      am &= am - 1;
      const int cl = __shfl(c, l);
      const double tl = rlane(t, l);
      if (lane == 0) h.add(cl, tl, false);
    }
  }
}

// wave 0: heap adds of T's nodes (z0 + k dz, x0 + k dx), k < n, in order, keys from T (64 loads
// per round trip)
AF_DEV void add_run(Lds* L, Heap& h, const XG& g, int z0, int x0, int dz, int dx, int n, int lane) {
  for (int k0 = 0; k0 < n; k0 += 64) {
    const int k = k0 + lane;
    double t = 0.0;
    if (k < n) t = gld(g.T + (long)(z0 + k * dz) * g.nx + (x0 + k * dx));
    const int m = min(64, n - k0);
    for (int l = 0; l < m; l++) {
      const double tl = rlane(t, l);
      const int z = z0 + (k0 + l) * dz, x = x0 + (k0 + l) * dx;
      if (lane == 0) h.add(g.loc(z, x), tl, false);
    }
  }
}

__global__ __launch_bounds__(kThreads) void fmm_exact_lds_kernel(BandParams P) {
  __shared__ Lds lds;
  Lds* L = &lds;
  const int src = blockIdx.x;
  crm::lds_init();
  if (src >= P.nsrc) return;
  BandSrc* B = P.src + src;
  const int tid = threadIdx.x, lane = tid & 63;
  const bool w0 = tid < 64;
  const DevModel& M = P.M;
  const int sg = P.sg, sgside = (sg - 1) / 2;
  const long isx = (long)sg * (long)rint((P.scx[src] - P.gox) / P.dnx);
  const long isz = (long)sg * (long)rint((P.scz[src] - P.goz) / P.dnz);
  const int nnz = P.nz, nnx = P.nx;
  __shared__ int err_s, ntr_s;
  if (tid == 0) err_s = 0;
  Heap h{L};
  Spec sp;
  sp.c = -1;
  sp.v = 0.0;
  sp.dirty = false;
  sp.vm = 0u;
  const double* pT = nullptr;
  int pnz = 0, pnx = 0, pisz = 0, pisx = 0;
  const int scales[2] = {9, 3};
  const int size1 = 2 * sg + (sg - 1) / 2, size2 = size1 + 3 * sg;
  for (int stg = 0; stg < 2; stg++) {
    __syncthreads();
    if (err_s) break;
    const int scale = scales[stg], size = stg == 0 ? size1 : size2;
    const int left = (int)max(0L, isx - size), right = (int)min((long)nnx - 1, isx + size);
    const int bottom = (int)max(0L, isz - size), top = (int)min((long)nnz - 1, isz + size);
    XG g;
    g.nz = scale * (top - bottom) + 1;
    g.nx = scale * (right - left) + 1;
    g.wz0 = g.wx0 = 0;
    g.wh = g.nz;
    g.ww = g.nx;
    if ((long)g.nz * g.nx > P.capS || (long)g.nz * g.nx > kCap) {
      if (tid == 0) err_s = 9;
      break;
    }
    g.T = gptr(B->Ts[stg]);
    g.mv = MatView{scale, (scale - 1) / 2, bottom, scale, (scale - 1) / 2, left, sg, sgside, 0, 0, 1};
    g.dnx = g.dnz = P.dnx / scale;
    const int isx_s = scale * (int)(isx - left), isz_s = scale * (int)(isz - bottom);
    if (stg == 1) classify(L, pnz, pnx, tid);  // the previous grid's statuses, before they are cleared
    __syncthreads();
    clear_state(L, g.nz * g.nx, tid);
    clear_grid(g.T, (long)g.nz * g.nx, tid);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's clear lands before wave 0 writes
    __syncthreads();
    h.ntr = 0;
    h.ndup = 0;
    h.livedup = 0;
    if (stg == 0) {
      // straight rays (:2223-2267; veln + angle, SURVEY B-D5), material of the source's fine cell
      const int side1 = (9 - 1) / 2 + 9 * ((sg - 1) / 2);
      const MatView fine{sg, sgside, 0, sg, sgside, 0, 1, 0, 0, 0, 1};
      const CellMat cs = cell_mat(M, fine, (int)isz, (int)isx);
      const int w = 2 * side1 + 1;
      for (int k = tid; k < w * w; k += kThreads) {
        const int i = k / w - side1, j = k % w - side1;
        if (0 <= isz_s + i && isz_s + i <= g.nz - 1 && 0 <= isx_s + j && isx_s + j <= g.nx - 1) {
          double angle = (j == 0) ? 90.0 : AF_ATAN((double)i / (double)j) * kRad2Deg;
          double eff = pymod(cs.veln + angle, 180);
          double velocity = (cs.velpn != 0 || cs.stif == nullptr) ? table_vel(M.gtab, M.ncol, eff, cs.velpn, cs.vm)
                                                                  : christoffel_group(cs.stif, eff, cs.vm);
          double length = g.dnx * sqrt((double)(i * i + j * j));
          gst(g.T + (long)(isz_s + i) * g.nx + isx_s + j, length / velocity);
          sset(L, (isz_s + i) * g.nx + isx_s + j, kSKnown);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (w0) {
        // window edges -> heap in the reference's order (:2277-2288)
        const int s1 = side1;
        const int xa = max(0, isx_s - s1), xb = min(g.nx - 1, isx_s + s1);
        const int za = max(0, isz_s - s1), zb = min(g.nz - 1, isz_s + s1);
        if (isz_s - s1 >= 0) add_run(L, h, g, isz_s - s1, xa, 0, 1, xb - xa + 1, lane);
        if (isz_s + s1 <= g.nz - 1) add_run(L, h, g, isz_s + s1, xa, 0, 1, xb - xa + 1, lane);
        if (isx_s - s1 >= 0) add_run(L, h, g, za, isx_s - s1, 1, 0, zb - za + 1, lane);
        if (isx_s + s1 <= g.nx - 1) add_run(L, h, g, za, isx_s + s1, 1, 0, zb - za + 1, lane);
      }
    } else if (w0) {
      handover(L, h, pT, pnz, pnx, pisz, pisx, g, isz_s, isx_s, lane);
    }
    if (AF_XL_TWO_ROLE) {
      if (tid == 0) {
        L->cmd = 0;
        L->done = 0;
        L->applied = 0;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // wave 0's grid stores before wave 1 reads them
      __syncthreads();
      if (w0) {
        const long long pops = heap_role(L, h, g, true, isx_s, isz_s, scale * size, 0.0, lane, B->ph);
        if (lane == 0) {
          B->steps[stg] = pops;
          if (h.err) err_s = h.err;
        }
      } else if (tid < 128) {
        relax_role(L, M, g, sp, lane, B->sub, B->ph);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (w0) {
      sp.c = -1;
      const long long pops = walk(L, h, M, g, true, isx_s, isz_s, scale * size, 0.0, sp, lane, B->sub, B->ph);
      if (lane == 0) {
        B->steps[stg] = pops;
        if (h.err) err_s = h.err;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    pT = g.T;
    pnz = g.nz;
    pnx = g.nx;
    pisz = isz_s;
    pisx = isx_s;
  }
  __syncthreads();
  // fine main grid (memset by the host: T NaN, S -1): the statuses of a window around the source
  // that holds the stage-2 hand-over and the prefix out to tstop
  const int Wh = size2 + P.exact_r + 8;  // tstop = (size2 + exact_r) dnx / vmax
  XG g;
  g.T = gptr(B->T);
  g.nz = nnz;
  g.nx = nnx;
  g.wz0 = (int)max(0L, isz - Wh);
  g.wx0 = (int)max(0L, isx - Wh);
  g.wh = (int)min((long)nnz - 1, isz + Wh) - g.wz0 + 1;
  g.ww = (int)min((long)nnx - 1, isx + Wh) - g.wx0 + 1;
  g.mv = MatView{sg, sgside, 0, sg, sgside, 0, 1, 0, 0, 0, 1};
  g.dnx = P.dnx;  // the coarse spacing on the fine grid (:2790; field divided by sg at the end)
  g.dnz = P.dnz;
  if (!err_s && (long)g.wh * g.ww > kCap && tid == 0) err_s = 9;
  if (!err_s) classify(L, pnz, pnx, tid);
  __syncthreads();
  int err = err_s;
  if (!err) {
    clear_state(L, g.wh * g.ww, tid);
    __syncthreads();
    if (w0) {
      h.ntr = 0;
      h.ndup = 0;
      h.livedup = 0;
      handover(L, h, pT, pnz, pnx, pisz, pisx, g, (int)isz, (int)isx, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (AF_XL_TWO_ROLE) {
      if (tid == 0) {
        L->cmd = 0;
        L->done = 0;
        L->applied = 0;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // wave 0's grid stores before wave 1 reads them
      __syncthreads();
      if (w0) {
        const long long pops = heap_role(L, h, g, false, 0, 0, 0, P.tstop, lane, B->ph);
        if (lane == 0) {
          B->steps[2] = pops;
          if (h.err) err_s = h.err;
        }
      } else if (tid < 128) {
        relax_role(L, M, g, sp, lane, B->sub, B->ph);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (w0) {
      sp.c = -1;
      const long long pops = walk(L, h, M, g, false, 0, 0, 0, P.tstop, sp, lane, B->sub, B->ph);
      if (lane == 0) {
        B->steps[2] = pops;
        if (h.err) err_s = h.err;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    err = err_s;
  }
  // outputs for the band kernel: the window as the written box, known nodes' status 0 in S,
  // close nodes (heap entries) -> S = heap index, Lin
  if (!err) {
    const int n = g.wh * g.ww;
    for (int k = tid; k < n; k += kThreads)
      if (sget(L, k) == kSKnown) gst(B->S + (long)g.gz(k) * nnx + g.gx(k), (int)kKnown);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) ntr_s = h.ntr;
    __syncthreads();
    const int nl = ntr_s;
    for (int k = 1 + tid; k <= nl && k <= P.capL; k += kThreads) {
      const unsigned e = L->ent[k];
      const int c = (int)(e & kNodeM);
      const int f = g.gz(c) * nnx + g.gx(c);
      if (!(e & kDupF)) gst(B->S + f, k);  // close: 1 + close-list slot
      gst(B->Lin + k - 1, f);
    }
    // a node with two entries: its S is the later entry's index, as fmm_exact.hip's in-order loop
    if (tid == 0 && h.ndup) {
      for (int k = 1; k <= nl && k <= P.capL; k++) {
        const unsigned e = L->ent[k];
        if (e & kDupF) gst(B->S + g.gz(e & kNodeM) * nnx + g.gx(e & kNodeM), k);
      }
    }
    if (tid == 0) {
      B->bbox[0] = g.wz0;
      B->bbox[1] = g.wz0 + g.wh - 1;
      B->bbox[2] = g.wx0;
      B->bbox[3] = g.wx0 + g.ww - 1;
      B->nl0 = nl;
      if (nl > P.capL) err = 2;
    }
  }
  if (tid == 0) B->err = err;
}

}  // namespace xl
}  // namespace af

// 1: the LDS walk holds subgrid sg's stage grids and the prefix window (else fmm_exact.hip)
extern "C" int af_exact_lds_fits(int sg, int exact_r) {
  const long size1 = 2L * sg + (sg - 1) / 2, size2 = size1 + 3L * sg;
  const long s1 = 9 * 2 * size1 + 1, s2 = 3 * 2 * size2 + 1, w = 2 * (size2 + exact_r + 8) + 1;
  const long d1 = (s1 - 1) / 3 + 1, d2 = (s2 - 1) / 3 + 1;
  return s1 * s1 <= af::xl::kCap && s2 * s2 <= af::xl::kCap && w * w <= af::xl::kCap && d1 * d1 <= af::xl::kDec &&
         d2 * d2 <= af::xl::kDec;
}

extern "C" hipError_t af_launch_exact_lds(const af::BandParams* P, hipStream_t stream) {
  hipLaunchKernelGGL(af::xl::fmm_exact_lds_kernel, dim3(P->nsrc), dim3(af::xl::kThreads), 0, stream, *P);
  return hipGetLastError();
}
