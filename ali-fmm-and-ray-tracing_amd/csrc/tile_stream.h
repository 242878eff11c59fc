// tile_stream.h — the host side of the band kernel's field streaming (alifmm_travel_into): the
// tile geometry of a launch and the copy threads' drain of the per-member queues.  Plain C++ (no
// HIP), shared by api.cpp and tests/stream_sim.cpp, which drives it against a CPU model of the
// kernel's side of the protocol (fmm_band_k.hip: tile_known / stage_tiles / publish_tiles /
// ring_space and the end flush).
//
// Protocol.  Band member m = source * K + k owns the stripes k, k + K, ... of its source; its own
// tiles are W = 2^wlog columns (one stripe) x TR = 2^trlog rows.  The member's i-th final tile is
// stored in slot i mod rslots of the member's ring (row-major, row pitch W) and then published as
// entry i of the member's queue: (i + 1) << 32 | tz * nstr + stripe.  The host copies entry i's
// tile out of its slot into the caller's field and then sets hcons[m] = i + 1; the kernel stores
// tile j only once hcons[m] >= j + 1 - rslots.  Every own tile is published exactly once.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

namespace af {
namespace ts {

constexpr int kListCap = 32;          // tiles a member stages per step (fmm_band_k.hip kTdCap)
constexpr int kOwnTileMax = 1024;     // own tiles per member with an LDS counter (kTileMax)
constexpr int kTileCellsMax = 32768;  // cells per tile (16-bit counters, 0xffff = published)
// slots per member: when a member asks for room for a list, the list it staged the step before is
// not yet published (the host cannot free those slots yet), so fewer slots than two lists could
// wait forever
constexpr int kRingSlots = 2 * kListCap;

struct Geometry {
  int K = 0, wlog = 0, trlog = 0, nstr = 0, ntz = 0, nz = 0, nx = 0, qcap = 0, rslots = 0;
  int W() const { return 1 << wlog; }
  int TR() const { return 1 << trlog; }
  int clog() const { return wlog + trlog; }
  // own tiles of member k of a source
  long expect(int k) const { return k < nstr ? (long)((nstr - k + K - 1) / K) * ntz : 0; }
};

// W x 2^trlog tiles with the fewest rows that keep every member's own tiles within kOwnTileMax;
// false when no such geometry exists (the fields are then copied after the launch)
inline bool plan(int K, int wlog, int fz, int fx, Geometry* g) {
  const int W = 1 << wlog, nstr = (fx + W - 1) / W, own = (nstr + K - 1) / K;
  int trlog = 2;
  while (trlog < 14 && (long)own * ((fz + (1 << trlog) - 1) >> trlog) > kOwnTileMax) trlog++;
  const int ntz = (fz + (1 << trlog) - 1) >> trlog;
  if ((long)own * ntz > kOwnTileMax || ((long)W << trlog) > kTileCellsMax) return false;
  g->K = K;
  g->wlog = wlog;
  g->trlog = trlog;
  g->nstr = nstr;
  g->ntz = ntz;
  g->nz = fz;
  g->nx = fx;
  g->qcap = own * ntz;
  g->rslots = kRingSlots;
  return true;
}

struct Buffers {
  const double* ring;             // [member][rslots][W << trlog]
  const unsigned long long* hq;   // [member][qcap]
  unsigned* hcons;                // [member]
};

inline void relax_cpu() {
#if defined(__x86_64__)
  for (int i = 0; i < 64; i++) __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}

// an idle pass over the queues: spin briefly, then yield, then sleep.  A member publishes a tile
// every ~0.4 ms at C4 and its ring holds 64, so a 50 us nap loses nothing; it keeps a context per
// GPU (update_parallel: one process, up to 8 teams) from spinning ~120 threads on a 16-CPU share
inline void idle_wait(int idle) {
  if (idle < 32) relax_cpu();
  else if (idle < 64) std::this_thread::yield();
  else std::this_thread::sleep_for(std::chrono::microseconds(50));
}

// Copy thread w of nw: the queues of members w, w + nw, ... of a launch of nsrc sources; each
// entry's tile goes from its slot into dst[source], row by row, and the slot is handed back.
// Ends when every expected tile has arrived, or once kernel_done() and a pass over the queues
// finds nothing new; the sources with missing tiles are marked in missing[].
template <class Done>
void drain(const Geometry& g, int nsrc, double* const* dst, const Buffers& b, int w, int nw, Done kernel_done,
           std::atomic<int>* missing) {
  struct Q {
    int m, pos;
    long expect;
  };
  std::vector<Q> qs;
  long remaining = 0;
  for (int m = w; m < nsrc * g.K; m += nw) {
    qs.push_back({m, 0, g.expect(m % g.K)});
    remaining += qs.back().expect;
  }
  const int W = g.W(), TR = g.TR();
  int quiet = 0, idle = 0;
  while (remaining > 0) {
    bool any = false;
    for (auto& q : qs) {
      while (q.pos < q.expect) {
        const unsigned long long v = __atomic_load_n(b.hq + (size_t)q.m * g.qcap + q.pos, __ATOMIC_ACQUIRE);
        if ((long)(v >> 32) != (long)q.pos + 1) break;
        const int t = (int)(unsigned)v, src = q.m / g.K;
        const int tz = t / g.nstr, st = t - tz * g.nstr;
        const int z0 = tz * TR, x0 = st * W;
        const int rows = std::min(TR, g.nz - z0), cols = std::min(W, g.nx - x0);
        double* d = dst[src];
        const double* sp = b.ring + (((size_t)q.m * g.rslots + q.pos % g.rslots) << g.clog());
        for (int r = 0; r < rows; r++)
          memcpy(d + (size_t)(z0 + r) * g.nx + x0, sp + (size_t)r * W, (size_t)cols * sizeof(double));
        q.pos++;
        __atomic_store_n(b.hcons + q.m, (unsigned)q.pos, __ATOMIC_RELEASE);  // the slot is free
        remaining--;
        any = true;
      }
    }
    if (any) {
      quiet = idle = 0;
      continue;
    }
    if (kernel_done()) {
      if (++quiet > 1) break;
    } else {
      idle_wait(idle++);
    }
  }
  for (auto& q : qs)
    if (q.pos < q.expect) missing[q.m / g.K].store(1);
}

}  // namespace ts
}  // namespace af
