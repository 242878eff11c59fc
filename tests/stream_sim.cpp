// CPU model of the band kernel's side of the field streaming (fmm_band_k.hip: tile_known,
// ring_space, stage_tiles, publish_tiles, the end flush), one thread per band member, against the
// library's own host side (csrc/tile_stream.h: plan, drain).  Every field must arrive intact in
// the caller's (non-consecutive) rows, every tile exactly once, with no deadlock, for bursts of
// completed tiles larger than a step's list (the overflow goes to the end flush) and grids that
// are not multiples of the tile.  Test infrastructure only (tests/test_host.py builds and runs it).
//   stream_sim NSRC K WLOG NZ NX SEED [RSLOTS WAIT_S]  -> "ok ..." or "FAIL ..." (exit status 1)
// (RSLOTS overrides the ring size: below 2 lists a member can wait for the host forever, which
// the model reports as a deadlock after WAIT_S seconds)
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "tile_stream.h"

using namespace af;

int main(int argc, char** argv) {
  if (argc < 7) return 2;
  const int nsrc = atoi(argv[1]), K = atoi(argv[2]), wlog = atoi(argv[3]), nz = atoi(argv[4]), nx = atoi(argv[5]);
  const unsigned seed = (unsigned)atoi(argv[6]);
  const int wait_s = argc > 8 ? atoi(argv[8]) : 20;
  ts::Geometry g;
  if (!ts::plan(K, wlog, nz, nx, &g)) {
    printf("ok no-geometry\n");
    return 0;
  }
  if (argc > 7) g.rslots = atoi(argv[7]);
  const size_t cells = (size_t)nz * nx, members = (size_t)nsrc * K;
  // the fields the kernel holds (distinct values per cell and source)
  std::vector<double> field(nsrc * cells);
  for (size_t i = 0; i < field.size(); i++) field[i] = 1.0 + (double)i * 1e-3;
  // the caller's stack: sources in reverse order, one spare row in front
  std::vector<double> stack((nsrc + 1) * cells, -7.0);
  std::vector<double*> dst(nsrc);
  for (int s = 0; s < nsrc; s++) dst[s] = stack.data() + (size_t)(nsrc - s) * cells;
  std::vector<double> ring(members * g.rslots << g.clog(), 0.0);
  std::vector<unsigned long long> hq(members * g.qcap, 0ull);
  std::vector<unsigned> hcons(members, 0u);
  std::atomic<int> done{0}, fail{0};
  std::unique_ptr<std::atomic<int>[]> missing(new std::atomic<int>[nsrc]);
  for (int s = 0; s < nsrc; s++) missing[s] = 0;

  auto member = [&](int m) {
    const int src = m / K, k = m % K;
    const int nown = k < g.nstr ? (g.nstr - k + K - 1) / K : 0, ntiles = nown * g.ntz;
    std::mt19937 rng(seed * 7919u + (unsigned)m);
    std::vector<int> order(ntiles);
    for (int o = 0; o < ntiles; o++) order[o] = o;
    std::shuffle(order.begin(), order.end(), rng);
    std::vector<char> published(ntiles, 0);
    std::vector<int> list[2];
    int qpos = 0, spos = 0, nst = 0, cons = 0;
    auto global = [&](int o) { return (o / nown) * g.nstr + k + (o % nown) * K; };
    auto ring_space = [&](int i0, int n) {
      const auto t0 = std::chrono::steady_clock::now();
      while (i0 + n - cons > g.rslots) {
        cons = (int)__atomic_load_n(&hcons[m], __ATOMIC_ACQUIRE);
        if (i0 + n - cons <= g.rslots) break;
        std::this_thread::yield();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(wait_s)) {  // a deadlock
          fail.store(1);
          cons = i0 + n;
        }
      }
    };
    auto stage = [&](const std::vector<int>& L, int n, int i0) {
      for (int j = 0; j < n; j++) {
        const int o = L[j], t = global(o), tz = t / g.nstr, st = t % g.nstr;
        const int z0 = tz * g.TR(), x0 = st * g.W();
        double* slot = ring.data() + (((size_t)m * g.rslots + (i0 + j) % g.rslots) << g.clog());
        for (int r = 0; r < g.TR() && z0 + r < nz; r++)
          for (int c = 0; c < g.W() && x0 + c < nx; c++)
            slot[(size_t)r * g.W() + c] = field[src * cells + (size_t)(z0 + r) * nx + x0 + c];
      }
    };
    auto publish = [&](std::vector<int>& L) {
      const int n = std::min((int)L.size(), ts::kListCap);
      for (int j = 0; j < n; j++) {
        __atomic_store_n(&hq[m * g.qcap + qpos + j], ((unsigned long long)(qpos + j + 1) << 32) | (unsigned)global(L[j]),
                         __ATOMIC_RELEASE);
        published[L[j]] = 1;
      }
      qpos += n;
      L.clear();
    };
    // steps: each completes a burst of tiles (0 .. 40: bursts past the list cap)
    size_t next = 0;
    for (int step = 0;; step++) {
      const int par = step & 1, prv = par ^ 1;
      spos += nst;  // P0h
      nst = std::min((int)list[prv].size(), ts::kListCap);
      if (nst) ring_space(spos, nst);
      if (!list[par].empty()) publish(list[par]);  // after the X1 drain
      if (nst) stage(list[prv], nst, spos);
      if (next >= order.size()) {                        // the band is done: the loop's break
        if (nst) publish(list[prv]);                     // end flush: the last staged list
        spos += nst;
        nst = 0;
        break;
      }
      const int burst = (int)(rng() % 41);  // accept: tiles completed this step
      for (int b = 0; b < burst && next < order.size(); b++) {
        if ((int)list[par].size() < ts::kListCap) list[par].push_back(order[next]);  // else: end flush
        next++;
      }
    }
    // end flush: the tiles never published, in windows of kListCap
    for (int base = 0; base < ntiles; base += ts::kListCap) {
      std::vector<int> L;
      for (int o = base; o < std::min(ntiles, base + ts::kListCap); o++)
        if (!published[o]) L.push_back(o);
      if (L.empty()) continue;
      ring_space(spos, (int)L.size());
      stage(L, (int)L.size(), spos);
      spos += (int)L.size();
      publish(L);
    }
  };

  const int nw = 3;
  const ts::Buffers b{ring.data(), hq.data(), hcons.data()};
  std::vector<std::thread> workers, kernel;
  for (int w = 0; w < nw; w++)
    workers.emplace_back([&, w] {
      ts::drain(g, nsrc, dst.data(), b, w, nw, [&] { return done.load() != 0; }, missing.get());
    });
  for (size_t m = 0; m < members; m++) kernel.emplace_back(member, (int)m);
  for (auto& t : kernel) t.join();
  done.store(1);
  for (auto& t : workers) t.join();
  long bad = 0;
  for (int s = 0; s < nsrc; s++) {
    if (missing[s].load()) bad++;
    for (size_t i = 0; i < cells; i++) bad += dst[s][i] != field[s * cells + i];
  }
  for (size_t i = 0; i < cells; i++) bad += stack[i] != -7.0;  // the spare row is untouched
  if (bad || fail.load()) {
    printf("FAIL bad=%ld deadlock=%d (trlog %d, rslots %d)\n", bad, fail.load(), g.trlog, g.rslots);
    return 1;
  }
  printf("ok nsrc=%d K=%d W=%d TR=%d tiles/member<=%d\n", nsrc, K, g.W(), g.TR(), g.qcap);
  return 0;
}
