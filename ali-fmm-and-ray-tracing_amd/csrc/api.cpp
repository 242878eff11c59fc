// api.cpp — host runtime behind include/alifmm.h (HIP, one context per GPU).
//
// Owns the HBM-resident model, the per-source work arena (status grid + band work lists) and
// the resident travel-time fields that the ray tracer reads without a host round trip.
// Sources are processed in launches of at most `batch` (and at most half the CUs: >= 2 band
// workgroups per source), all workgroups of a launch co-resident.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/alifmm.h"
#include "context.h"
#include "kernels.h"
#include "tile_stream.h"

extern char** environ;

static void free_ray_bufs(alifmm_ctx* c) {
  auto& b = c->rb;
  for (void* p : {(void*)b.rx, (void*)b.ry, (void*)b.t, (void*)b.len, (void*)b.flags, (void*)b.jobs, (void*)b.off})
    if (p) (void)hipFree(p);
  b = alifmm_ctx::RayBufs();
}
// points kept by alifmm_find_rays(..., ALIFMM_KEEP_RAYS) for alifmm_take_rays
static void release_kept_rays(alifmm_ctx* c) {
  for (auto& k : c->kept_dev) dfree(k.d);
  c->kept_dev.clear();
  std::vector<std::vector<double>>().swap(c->kept_rays);
  c->kept_pts = 0;
}
static void free_arena(Arena& a) {
  dfree(a.S); dfree(a.lists); dfree(a.dlists); dfree(a.Ts); dfree(a.Ss); dfree(a.srcs); dfree(a.ho); dfree(a.jobs);
  dfree(a.rimc); dfree(a.rimt); dfree(a.kx); dfree(a.Tb); dfree(a.Sb);
  dfree(a.dscx); dfree(a.dscz);
  a = Arena();
}

// ---- host-side velocity maximum (for the band width) ----
static double pymod(double a, double b) {
  double m = std::fmod(a, b);
  if (m != 0.0) {
    if ((b < 0) != (m < 0)) m += b;
  } else {
    m = std::copysign(0.0, b);
  }
  return m;
}
static double christoffel_group_host(const double* s, double eff, double vm) {
  double e90 = pymod(eff, 90);
  if (e90 < 0.01 || e90 > 90 - 0.01) {
    double lam = (std::fabs(pymod(eff, 180) - 90) < 1) ? s[2] : s[0];
    return 1000 * vm * std::sqrt(lam / s[4]);
  }
  double tan_ang = std::tan(eff * M_PI / 180.0);
  double A = s[0] + s[2] - 2 * s[3], B = (s[1] + s[3]) * (tan_ang - 1 / tan_ang), C = s[0] - s[2];
  double disc = B * B + A * A - C * C;
  double pa = eff < 90 ? pymod(std::atan((-B - std::sqrt(disc)) / (C - A)), M_PI)
                       : pymod(std::atan((-B + std::sqrt(disc)) / (C - A)), M_PI);
  double lam = 0.5 * (std::cos(2 * pa) * (s[0] - s[3]) + std::sin(2 * pa) * (s[1] + s[3]) * tan_ang + s[0] + s[3]);
  return 1000 * vm * std::sqrt(lam / s[4]) / std::cos(eff * M_PI / 180.0 - pa);
}

// material-id table capacity (the band kernel stages <= kMatLds of them in LDS)
static const int kMaxMatIds = 4096;
// plane-search candidates per ray the ray kernel holds (rays.hip kMaxCand)
static const int kMaxRayCand = 256;
// ray point buffers larger than this are freed at the end of each alifmm_find_rays call
static const size_t kRayBufKeepBytes = (size_t)1 << 30;

// host copies up to this size go straight to pageable memory while the pinned ring is unallocated
static const size_t kSmallD2H = (size_t)64 << 20;
// contexts alive in this process (copy teams share the process's CPU share between them)
static std::atomic<int> g_live_ctx{0};

// ---- set_model's per-cell passes over the host threads ----
// the process's CPU share (OMP_NUM_THREADS on the GPU box, else the hardware's, at most 32)
static int host_threads() {
  int n = (int)std::max(1u, std::thread::hardware_concurrency());
  if (const char* e = getenv("OMP_NUM_THREADS")) {
    const int v = atoi(e);
    if (v >= 1) n = v;
  }
  // contexts that upload models at the same time (update_parallel: one per GPU) share the share
  return std::max(1, std::min(n, 32) / std::max(1, g_live_ctx.load()));
}
// fn(chunk, lo, hi) over nch contiguous chunks of [0, n), one thread each
// (serially below min_n items: the default suits per-cell passes; row passes give a smaller one)
static void for_chunks(size_t n, int nch, const std::function<void(int, size_t, size_t)>& fn,
                       size_t min_n = 65536) {
  if (nch <= 1 || n < min_n) {
    fn(0, 0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int c = 0; c < nch; c++) th.emplace_back(fn, c, n * c / nch, n * (c + 1) / nch);
  for (auto& t : th) t.join();
}
// Distinct keys of cells [0, n) (key(i)), numbered in order of first occurrence — the serial scan's
// numbering: each chunk numbers its own keys (runs of equal keys skip the map), then the chunks'
// keys are merged in chunk order and the ids remapped.  ids[i]: the cell's key id; order: the keys
// by id.  False when a chunk or the merge finds more than max_keys keys (ids then unusable).
template <class Key, class KeyFn>
static bool unique_ids(size_t n, int nth, KeyFn key, std::vector<int>& ids, std::vector<Key>& order,
                       size_t max_keys) {
  const int nch = n < 65536 ? 1 : nth;
  std::vector<std::vector<Key>> local(nch);
  std::vector<char> over(nch, 0);
  ids.resize(n);
  for_chunks(n, nch, [&](int c, size_t lo, size_t hi) {
    std::map<Key, int> uniq;
    Key last{};
    int last_id = -1;
    for (size_t i = lo; i < hi; i++) {
      const Key k = key(i);
      if (last_id >= 0 && k == last) {
        ids[i] = last_id;
        continue;
      }
      auto it = uniq.find(k);
      int id;
      if (it == uniq.end()) {
        id = (int)local[c].size();
        if ((size_t)id >= max_keys) {
          over[c] = 1;
          return;
        }
        uniq.emplace(k, id);
        local[c].push_back(k);
      } else {
        id = it->second;
      }
      ids[i] = id;
      last = k;
      last_id = id;
    }
  });
  for (int c = 0; c < nch; c++)
    if (over[c]) return false;
  std::map<Key, int> glob;
  std::vector<std::vector<int>> remap(nch);
  for (int c = 0; c < nch; c++) {
    for (const Key& k : local[c]) {
      auto it = glob.find(k);
      int g;
      if (it == glob.end()) {
        g = (int)order.size();
        if ((size_t)g >= max_keys) return false;
        glob.emplace(k, g);
        order.push_back(k);
      } else {
        g = it->second;
      }
      remap[c].push_back(g);
    }
  }
  for_chunks(n, nch, [&](int c, size_t lo, size_t hi) {
    const std::vector<int>& r = remap[c];
    for (size_t i = lo; i < hi; i++) ids[i] = r[ids[i]];
  });
  return true;
}

extern "C" {

const char* alifmm_version(void) { return "alifmm-mi355x 0.1 (gfx950)"; }

int alifmm_device_count(int* n) {
  int k = 0;
  hipError_t e = hipGetDeviceCount(&k);
  if (e != hipSuccess) k = 0;
  *n = k;
  return e == hipSuccess ? ALIFMM_OK : ALIFMM_E_HIP;
}

int alifmm_ctx_create(int device, alifmm_ctx** out) {
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ALIFMM_E_HIP;
  if (device < 0 || device >= n) return ALIFMM_E_ARG;
  alifmm_ctx* ctx = new alifmm_ctx();
  ctx->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return ALIFMM_E_HIP;
  }
  for (auto& e : ctx->ev) (void)hipEventCreate(&e);
  if (hipStreamCreateWithFlags(&ctx->fill, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_fill, hipEventDisableTiming) != hipSuccess) {
    ctx->fill = nullptr;  // fills then stay on the main stream
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->n_cu = prop.multiProcessorCount;
  // band kernel launch: cooperative (gang-scheduled: every member resident whatever else runs on
  // the device) by default; under rocprofv3 a plain launch after a residency check, because the
  // runtime's teardown of the cooperative queue at exit crashed after the profiler had finalised
  // (the plain path assumes exclusive use of the device; a member that never sees its peers stops
  // at the exchange's spin limit, error 7, and the chunk is re-run with a cooperative launch)
  ctx->coop = 1;
  for (char** e = environ; e && *e; e++)
    if (!strncmp(*e, "ROCPROF", 7) || !strncmp(*e, "ROCP_", 5)) ctx->coop = 0;
  g_live_ctx++;
  *out = ctx;
  return ALIFMM_OK;
}

static void free_model(alifmm_ctx* c) {
  dfree(c->d_veln); dfree(c->d_vm); dfree(c->d_velpn); dfree(c->d_sidx); dfree(c->d_stab); dfree(c->d_gtab);
  dfree(c->d_ptab); dfree(c->d_mid); dfree(c->d_mid8); dfree(c->d_mid8b); dfree(c->d_mtab); dfree(c->d_mslo);
  c->d_mid = nullptr;
  c->d_mid8 = nullptr;
  c->d_mid8b = nullptr;
  c->d_mtab = nullptr;
  c->d_mslo = nullptr;
  c->nmat = 0;
  c->d_veln = c->d_vm = c->d_stab = c->d_gtab = c->d_ptab = nullptr;
  c->d_velpn = c->d_sidx = nullptr;
  c->have_model = false;
}

static void free_stream_bufs(alifmm_ctx* ctx);

int alifmm_release_fields(alifmm_ctx* ctx) {
  if (!ctx) return ALIFMM_E_ARG;
  (void)hipSetDevice(ctx->device);
  for (auto& f : ctx->fields) dfree(f.d);
  ctx->fields.clear();
  free_ray_bufs(ctx);  // the ray tracer's point buffers (chunk x max_pts per coordinate) go with the fields
  release_kept_rays(ctx);
  free_stream_bufs(ctx);  // the pinned staging of streamed fields too
  return ALIFMM_OK;
}

static void destroy_team(alifmm_ctx* ctx);

int alifmm_ctx_destroy(alifmm_ctx* ctx) {
  if (!ctx) return ALIFMM_OK;
  g_live_ctx--;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  destroy_team(ctx);
  alifmm_release_fields(ctx);
  free_arena(ctx->arena);
  dfree(ctx->ho_all);
  dfree(ctx->jobs_all);
  ctx->ho_all = nullptr;
  ctx->jobs_all = nullptr;
  ctx->ho_last = nullptr;
  free_ray_bufs(ctx);
  for (int b = 0; b < alifmm_ctx::kPinBufs; b++) {
    if (ctx->pin[b]) (void)hipHostFree(ctx->pin[b]);
    if (ctx->pin_ev[b]) (void)hipEventDestroy(ctx->pin_ev[b]);
  }
  free_model(ctx);
  for (auto& e : ctx->ev) if (e) (void)hipEventDestroy(e);
  if (ctx->fill) {
    (void)hipStreamSynchronize(ctx->fill);
    (void)hipStreamDestroy(ctx->fill);
  }
  if (ctx->ev_fill) (void)hipEventDestroy(ctx->ev_fill);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return ALIFMM_OK;
}

const char* alifmm_last_error(alifmm_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

int alifmm_set_option(alifmm_ctx* ctx, const char* name, double value) {
  if (!ctx || !name) return ALIFMM_E_ARG;
  if (!strcmp(name, "cdelta") && value > 0) {
    ctx->cdelta = value;
    ctx->cdelta_set = true;
  }
  else if (!strcmp(name, "r0") && value >= 0) ctx->r0 = value;
  else if (!strcmp(name, "cdelta_far") && value >= 0) ctx->cdelta_far = value;
  else if (!strcmp(name, "r_far") && value >= 0) ctx->r_far = value;
  else if (!strcmp(name, "far_sg") && value >= 0 && value == (int)value) ctx->far_sg = (int)value;
  else if (!strcmp(name, "batch") && value >= 1) ctx->batch = (int)value;
  else if (!strcmp(name, "prof")) ctx->prof = value != 0;
  else if (!strcmp(name, "coop")) ctx->coop = value != 0;
  else if (!strcmp(name, "exact_r") && value >= 0 && value <= 48) ctx->exact_r = (int)value;
  else if (!strcmp(name, "exact_lds")) ctx->exact_lds = value != 0;
  else if (!strcmp(name, "stream_out")) ctx->stream_out = value != 0;
  else if (!strcmp(name, "members") && value >= 0 && value <= af::kMaxK && value == (int)value)
    ctx->members = (int)value;
  else if (!strcmp(name, "stripe_log") && (value == 0 || (value >= 3 && value <= 12))) ctx->stripe_log = (int)value;
  else return fail(ctx, ALIFMM_E_ARG, "unknown option or bad value: %s=%g", name, value);
  return ALIFMM_OK;
}

int alifmm_get_option(alifmm_ctx* ctx, const char* name, double* value) {
  if (!ctx || !name || !value) return ALIFMM_E_ARG;
  if (!strcmp(name, "cdelta")) *value = band_cdelta(ctx);  // in force for the resident model
  else if (!strcmp(name, "r0")) *value = ctx->r0;
  else if (!strcmp(name, "cdelta_far")) *value = band_cdelta_far(ctx);
  else if (!strcmp(name, "mat_jump")) *value = ctx->mat_jump;
  else if (!strcmp(name, "r_far")) *value = ctx->r_far;
  else if (!strcmp(name, "far_sg")) *value = ctx->far_sg;
  else if (!strcmp(name, "batch")) *value = ctx->batch;
  else if (!strcmp(name, "exact_r")) *value = ctx->exact_r;
  else if (!strcmp(name, "exact_lds")) *value = ctx->exact_lds;
  else if (!strcmp(name, "stream_out")) *value = ctx->stream_out;
  else if (!strcmp(name, "stream_tail_ms")) *value = ctx->t_stream_tail;      // last travel with a host destination
  else if (!strcmp(name, "stream_fallback")) *value = (double)ctx->stream_fallback;
  else if (!strcmp(name, "exact_redo")) *value = (double)ctx->exact_redo;
  else if (!strcmp(name, "prof")) *value = ctx->prof;
  else if (!strcmp(name, "coop")) *value = ctx->coop;
  else if (!strcmp(name, "members")) *value = ctx->members;
  else if (!strcmp(name, "stripe_log")) *value = ctx->stripe_log;
  else if (!strcmp(name, "last_k")) *value = ctx->last_k;
  else if (!strcmp(name, "n_cu")) *value = ctx->n_cu;
  else if (!strcmp(name, "vmax")) *value = ctx->vmax;  // model's fastest speed (set_model; the exact-walk stop)
  else if (!strcmp(name, "nmat")) *value = ctx->nmat;  // distinct material records (0: past the id table)
  else if (!strcmp(name, "ray_lanes")) *value = ctx->last_ray_lanes;  // lanes per ray, last find_rays
  else if (!strcmp(name, "ray_waves_per_simd")) *value = af_ray_waves_per_simd();  // ray kernel occupancy target
  // timings of the last alifmm_find_rays / alifmm_take_rays call (ms): ray kernel and point-packing
  // kernel (HIP events, summed over the launches), the whole call, and the kept points' copy-out
  else if (!strcmp(name, "ray_kernel_ms")) *value = ctx->t_ray_kernel;
  else if (!strcmp(name, "ray_pack_ms")) *value = ctx->t_ray_pack;
  else if (!strcmp(name, "find_rays_ms")) *value = ctx->t_find_rays;
  else if (!strcmp(name, "take_rays_ms")) *value = ctx->t_take_rays;
  else return fail(ctx, ALIFMM_E_ARG, "unknown option: %s", name);
  return ALIFMM_OK;
}

static af::DevModel dev_model(const alifmm_ctx* c);
int alifmm_copy_fields(alifmm_ctx* ctx, int first_slot, int n, double* dst, int dst_kind, double* gbps);

int alifmm_set_model(alifmm_ctx* ctx, int nnz, int nnx, const double* veln, const int64_t* velpn,
                     const double* vel_map, const int64_t* stif_den, const double* group_tab,
                     const double* phase_tab, int ncol, double dnx, double dnz, double gox, double goz) {
  if (!ctx || nnz < 2 || nnx < 2 || !veln || !velpn || !vel_map || !group_tab || !phase_tab || ncol < 1 ||
      ncol >= 32768)  // (the init kernels pack velpn and ncol in one int)
    return fail(ctx, ALIFMM_E_ARG, "set_model: bad arguments");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  // everything that can reject the model is checked before the resident model is released, so a
  // rejected call leaves the previous model usable
  const size_t n = (size_t)nnz * nnx;
  const int nth = host_threads();
  std::vector<int> vp(n);
  {
    std::vector<size_t> bad(std::max(1, nth), SIZE_MAX);  // per chunk: the first bad cell
    for_chunks(n, nth, [&](int c, size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; i++) {
        if (velpn[i] < 0 || velpn[i] >= ncol) {
          bad[c] = i;
          return;
        }
        vp[i] = (int)velpn[i];
      }
    });
    for (size_t b : bad)
      if (b != SIZE_MAX)
        return fail(ctx, ALIFMM_E_ARG, "velpn[%zu]=%lld outside the table", b, (long long)velpn[b]);
  }
  // unique stiffness rows (numbered in order of first occurrence)
  std::vector<int> sidx;
  std::vector<double> stab;
  if (stif_den) {
    std::vector<std::array<int64_t, 5>> rows;
    unique_ids<std::array<int64_t, 5>>(
        n, nth,
        [&](size_t i) {
          std::array<int64_t, 5> row;
          for (int k = 0; k < 5; k++) row[k] = stif_den[5 * i + k];
          return row;
        },
        sidx, rows, SIZE_MAX);
    for (const auto& row : rows)
      for (int k = 0; k < 5; k++) stab.push_back((double)row[k]);
  }
  // maximum group velocity over the model (band width scale)
  double vmax = 0;
  {
    std::vector<double> colmax(ncol, 0.0);
    for (int c = 0; c < ncol; c++)
      for (int a = 0; a <= 180; a++) colmax[c] = std::max(colmax[c], group_tab[a * ncol + c]);
    const int nrow = (int)stab.size() / 5;
    std::vector<double> rowmax(nrow, 0.0);
    for (int r = 0; r < nrow; r++)
      for (int k = 0; k <= 3600; k++)
        rowmax[r] = std::max(rowmax[r], christoffel_group_host(&stab[5 * r], 0.05 * k, 1.0));
    for (size_t i = 0; i < n; i++) {
      double v = (vp[i] != 0 || !stif_den) ? colmax[vp[i]] * vel_map[i] : rowmax[sidx[i]] * vel_map[i];
      if (std::isfinite(v)) vmax = std::max(vmax, v);
    }
  }
  if (!(vmax > 0)) return fail(ctx, ALIFMM_E_ARG, "model has no positive velocity");
  // material-interface density (band_cdelta): 4-neighbour pairs whose (veln, vel_map, velpn,
  // stiffness row) differ, over all pairs; rows spread over the host threads
  double jump = 0.0;
  {
    std::vector<long> cnt(std::max(1, nth), 0);
    auto same = [&](size_t a, size_t b) {
      return !memcmp(&veln[a], &veln[b], 8) && !memcmp(&vel_map[a], &vel_map[b], 8) && vp[a] == vp[b] &&
             (!stif_den || sidx[a] == sidx[b]);
    };
    for_chunks((size_t)nnz, n < 65536 ? 1 : std::min(nth, nnz), [&](int c, size_t z0, size_t z1) {
      long k = 0;
      for (size_t z = z0; z < z1; z++)
        for (int x = 0; x < nnx; x++) {
          const size_t i = z * nnx + x;
          if (x + 1 < nnx && !same(i, i + 1)) k++;
          if (z + 1 < (size_t)nnz && !same(i, i + nnx)) k++;
        }
      cnt[c] = k;
    }, 1);
    long k = 0;
    for (long v : cnt) k += v;
    jump = (double)k / (double)((long)(nnz - 1) * nnx + (long)nnz * (nnx - 1));
  }
  free_model(ctx);
  HIPCHK(dalloc(&ctx->d_veln, n));
  HIPCHK(dalloc(&ctx->d_vm, n));
  HIPCHK(dalloc(&ctx->d_velpn, n));
  HIPCHK(dalloc(&ctx->d_gtab, (size_t)361 * ncol));
  HIPCHK(dalloc(&ctx->d_ptab, (size_t)361 * ncol));
  HIPCHK(hipMemcpy(ctx->d_veln, veln, n * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ctx->d_vm, vel_map, n * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ctx->d_velpn, vp.data(), n * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ctx->d_gtab, group_tab, (size_t)361 * ncol * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ctx->d_ptab, phase_tab, (size_t)361 * ncol * 8, hipMemcpyHostToDevice));
  if (stif_den) {
    HIPCHK(dalloc(&ctx->d_sidx, n));
    HIPCHK(dalloc(&ctx->d_stab, stab.size()));
    HIPCHK(hipMemcpy(ctx->d_sidx, sidx.data(), n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ctx->d_stab, stab.data(), stab.size() * 8, hipMemcpyHostToDevice));
  }
  // distinct (veln, vel_map, velpn, stiffness row) records -> per-cell material ids
  {
    std::vector<af::MatRec> recs;
    std::vector<int> mid;
    std::vector<std::array<int64_t, 4>> keys;
    const bool ok = unique_ids<std::array<int64_t, 4>>(
        n, nth,
        [&](size_t i) {
          std::array<int64_t, 4> key;
          memcpy(&key[0], &veln[i], 8);
          memcpy(&key[1], &vel_map[i], 8);
          key[2] = vp[i];
          key[3] = stif_den ? sidx[i] : -1;
          return key;
        },
        mid, keys, (size_t)kMaxMatIds);
    for (const auto& key : keys) {
      af::MatRec m;
      memcpy(&m.veln, &key[0], 8);
      memcpy(&m.vm, &key[1], 8);
      m.velpn = (int)key[2];
      m.sidx = (int)key[3];
      recs.push_back(m);
    }
    if (ok) {
      HIPCHK(dalloc(&ctx->d_mid, n));
      HIPCHK(dalloc(&ctx->d_mtab, recs.size()));
      HIPCHK(hipMemcpy(ctx->d_mid, mid.data(), n * 4, hipMemcpyHostToDevice));
      if (recs.size() <= 256) {  // byte ids: 4x fewer lines per material gather in the band kernels
        std::vector<unsigned char> m8(n);
        for_chunks(n, nth, [&](int, size_t lo, size_t hi) {
          for (size_t i = lo; i < hi; i++) m8[i] = (unsigned char)mid[i];
        });
        HIPCHK(dalloc(&ctx->d_mid8, n));
        HIPCHK(hipMemcpy(ctx->d_mid8, m8.data(), n, hipMemcpyHostToDevice));
        // the same ids in 8 x 16 bricks (one 128-byte line each) for the band kernel's subgrid-1 view
        const int bp = (nnx + 15) / 16, bz = (nnz + 7) / 8;
        std::vector<unsigned char> mb((size_t)128 * bp * bz, 0);
        for_chunks((size_t)bz, std::min(nth, bz), [&](int, size_t b0, size_t b1) {  // brick rows
          for (int z = (int)b0 * 8; z < std::min(nnz, (int)b1 * 8); z++)
            for (int x = 0; x < nnx; x++)
              mb[(((size_t)(z >> 3) * bp + (x >> 4)) << 7) | ((z & 7) << 4) | (x & 15)] = m8[(size_t)z * nnx + x];
        }, n < 65536 ? SIZE_MAX : 1);
        HIPCHK(dalloc(&ctx->d_mid8b, mb.size()));
        HIPCHK(hipMemcpy(ctx->d_mid8b, mb.data(), mb.size(), hipMemcpyHostToDevice));
        ctx->mid8b_pitch = bp;
      }
      HIPCHK(hipMemcpy(ctx->d_mtab, recs.data(), recs.size() * sizeof(af::MatRec), hipMemcpyHostToDevice));
      ctx->nmat = (int)recs.size();
    }
  }
  ctx->nstab = (int)stab.size() / 5;
  ctx->nz0 = nnz;
  ctx->nx0 = nnx;
  ctx->ncol = ncol;
  ctx->dnx = dnx;
  ctx->dnz = dnz;
  ctx->gox = gox;
  ctx->goz = goz;
  ctx->vmax = vmax;
  ctx->mat_jump = jump;
  if (ctx->nmat > 0) {  // fouds18_A() slownesses per material (band kernels' fallback)
    HIPCHK(dalloc(&ctx->d_mslo, 8 * (size_t)ctx->nmat));
    const af::DevModel M = dev_model(ctx);
    HIPCHK(af_launch_mat_slowness(&M, ctx->d_mslo, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  ctx->have_model = true;
  return ALIFMM_OK;
}

int alifmm_field_shape(alifmm_ctx* ctx, int subgrid, int* fnz, int* fnx) {
  if (!ctx || !ctx->have_model || subgrid < 1 || subgrid % 2 == 0)
    return fail(ctx, ALIFMM_E_ARG, "field_shape: no model or even subgrid %d", subgrid);
  *fnz = subgrid * (ctx->nz0 - 1) + 1;
  *fnx = subgrid * (ctx->nx0 - 1) + 1;
  return ALIFMM_OK;
}

static af::DevModel dev_model(const alifmm_ctx* c) {
  af::DevModel M;
  M.nz0 = c->nz0;
  M.nx0 = c->nx0;
  M.veln = c->d_veln;
  M.velpn = c->d_velpn;
  M.vm = c->d_vm;
  M.sidx = c->d_sidx;
  M.stab = c->d_stab;
  M.nstab = c->nstab;
  M.mid = c->d_mid;
  M.mid8 = c->d_mid8;
  M.mid8b = c->d_mid8b;
  M.mid8b_pitch = c->mid8b_pitch;
  M.mtab = c->d_mtab;
  M.nmat = c->nmat;
  M.mslo = c->d_mslo;
  M.gtab = c->d_gtab;
  M.ptab = c->d_ptab;
  M.ncol = c->ncol;
  return M;
}

// scells: cells of the row-major status S (fmm_exact_kernel's region and the mode-1 hand-over:
// subgrid > 1 only; 0 at subgrid 1, where the band kernel keeps its status in the bricked Sb)
static int ensure_arena(alifmm_ctx* ctx, int nsrc, long cells, long scells, long capL, long capC, long capS, int K,
                        long capR, long ecells, long tbc, long sbc) {
  Arena& a = ctx->arena;
  if (a.nsrc >= nsrc && a.cells >= cells && a.scells >= scells && a.capL >= capL && a.capC >= capC &&
      a.capS >= capS && a.K >= K && a.capR >= capR && a.ecells >= ecells && a.tbc >= tbc && a.sbc >= sbc)
    return ALIFMM_OK;
  if (ctx->ho_last == a.ho) {  // init profile of a chunk whose arena goes away
    ctx->ho_last = nullptr;
    ctx->n_ho_last = 0;
  }
  free_arena(a);
  a.nsrc = nsrc;
  a.cells = cells;
  a.scells = scells;
  a.capL = capL;
  a.capC = capC;
  a.capS = capS;
  a.K = K;
  a.capR = capR;
  a.ecells = ecells;
  a.tbc = tbc;
  a.sbc = sbc;
  HIPCHK(dalloc(&a.Tb, (size_t)nsrc * tbc));
  HIPCHK(dalloc(&a.Sb, (size_t)nsrc * sbc));
  if (scells > 0) HIPCHK(dalloc(&a.S, (size_t)nsrc * scells));
  HIPCHK(dalloc(&a.lists, (size_t)nsrc * (4 * capL + 6 * capC)));
  HIPCHK(dalloc(&a.dlists, (size_t)nsrc * (capL + 2 * capC)));
  if (K > 1) {
    HIPCHK(dalloc(&a.rimc, (size_t)nsrc * K * 2 * capR));
    HIPCHK(dalloc(&a.rimt, (size_t)nsrc * K * 2 * capR));
  }
  HIPCHK(dalloc(&a.kx, nsrc));
  if (capS > 0) {
    HIPCHK(dalloc(&a.Ts, (size_t)nsrc * 2 * capS));
    HIPCHK(dalloc(&a.Ss, (size_t)nsrc * 2 * capS));
  }
  HIPCHK(dalloc(&a.srcs, nsrc));
  HIPCHK(dalloc(&a.ho, nsrc));
  HIPCHK(dalloc(&a.jobs, nsrc));
  HIPCHK(dalloc(&a.dscx, nsrc));
  HIPCHK(dalloc(&a.dscz, nsrc));
  return ALIFMM_OK;
}

int af_ensure_field(alifmm_ctx* ctx, int slot, int sg, int fz, int fx, long extra_cells) {
  if ((int)ctx->fields.size() <= slot) ctx->fields.resize(slot + 1);
  Field& f = ctx->fields[slot];
  const size_t bytes = (size_t)fz * fx * sizeof(double), need = bytes + (size_t)extra_cells * sizeof(double);
  if (f.d && f.alloc < need) {
    dfree(f.d);
    f.d = nullptr;
  }
  if (!f.d) {
    HIPCHK(hipMalloc((void**)&f.d, need));
    f.alloc = need;
  }
  f.bytes = bytes;
  f.sg = sg;
  f.nz = fz;
  f.nx = fx;
  return ALIFMM_OK;
}

// members per source of the band kernel: the largest K <= kMaxK whose grid (nsrc padded to 8, times
// K workgroups, af_band_wgs_per_cu() of them per CU) is co-resident, with >= 2 stripes per member
// (option "members" forces a value, still capped by residency)
static int choose_members(const alifmm_ctx* ctx, int n, int fx) {
  const int by_cu = std::max(1, ctx->n_cu * af_band_wgs_per_cu() / (8 * ((n + 7) / 8)));
  if (ctx->members > 0) return std::max(1, std::min(ctx->members, by_cu));
  // >= 2 stripes per member at the stripe width the member count selects
  auto stripes = [&](int k) { return (long)(fx + (1 << (k >= 8 ? 4 : 6)) - 1) >> (k >= 8 ? 4 : 6); };
  int K = std::min(af::kMaxK, by_cu);
  while (K > 1 && 2L * K > stripes(K)) K--;
  return K;
}

// subgrid-1 source init (fmm_init_kernel) of n sources into ho (jobs: device scratch of n InitJobs)
static int launch_source_init(alifmm_ctx* ctx, int n, const double* scx, const double* scz, af::InitJob* djobs,
                              af::HandoverOut* ho) {
  std::vector<af::InitJob> jobs(n);
  for (int i = 0; i < n; i++) {
    jobs[i].isx = (long)std::nearbyint((scx[i] - ctx->gox) / ctx->dnx);
    jobs[i].isz = (long)std::nearbyint((scz[i] - ctx->goz) / ctx->dnz);
    jobs[i].dnx = ctx->dnx;
    jobs[i].dnz = ctx->dnz;
    jobs[i].exact_r = ctx->exact_r;
    jobs[i].tstop = ctx->exact_r * ctx->dnx / ctx->vmax;
    if (jobs[i].isx < 0 || jobs[i].isx >= ctx->nx0 || jobs[i].isz < 0 || jobs[i].isz >= ctx->nz0)
      return fail(ctx, ALIFMM_E_ARG, "source %d (%g, %g) outside the grid", i, scx[i], scz[i]);
  }
  af::DevModel M = dev_model(ctx);
  HIPCHK(hipMemcpyAsync(djobs, jobs.data(), sizeof(af::InitJob) * n, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(af_launch_init(&M, djobs, n, ho, ctx->stream));
  return ALIFMM_OK;
}

// alifmm_travel_into / alifmm_travel with a host destination: the caller's field of each source of
// a chunk, and the state of streaming them out of the band kernel (subgrid 1)
struct StreamOut {
  double* const* dst = nullptr;  // per source of the chunk
  int n = 0;
  bool active = false;  // the band launch streams (stream_setup)
  af::ts::Geometry g;
  std::atomic<int> kernel_done{0};
  std::unique_ptr<std::atomic<int>[]> missing;  // per source: a tile never arrived (copied after)
};
static int stream_setup(alifmm_ctx* ctx, StreamOut* so, int n, int K, int wlog, int fz, int fx);
static void stream_start(alifmm_ctx* ctx, StreamOut* so);
static void stream_finish(alifmm_ctx* ctx, StreamOut* so);

// travel_chunk: a plain band launch whose members were not all resident (another process held CUs);
// alifmm_travel re-runs the chunk once with a cooperative launch
static const int kRetryCoop = -100;

// one chunk of sources; returns ALIFMM_E_CAPACITY when a work list overflowed
static int travel_chunk(alifmm_ctx* ctx, int sg, int n, const double* scx, const double* scz, int first_slot, int fz,
                        int fx, float* ms_init, float* ms_band, const af::HandoverOut* pre_ho = nullptr,
                        StreamOut* so = nullptr) {
  const long cells = (long)fz * fx;
  long capL = std::min(cells, std::max(65536L, cells / 8) * ctx->cap_scale);
  long capC = capL;
  long capS = 0;
  if (sg > 1) {
    long s1 = 9L * 2 * (2L * sg + (sg - 1) / 2) + 1;             // stage-1 grid side (x9)
    long s2 = 3L * 2 * (2L * sg + (sg - 1) / 2 + 3L * sg) + 1;  // stage-2 grid side (x3)
    capS = std::max(s1 * s1, s2 * s2);
    capL = std::max(capL, std::min(capS, 262144L));
    capC = capL;
  }
  // band kernel: members per source and the stripe geometry (KGeom)
  const int K = choose_members(ctx, n, fx);
  // stripe width: 16 columns at 16 members, 32 at 8, 64 below (C4 sweeps, profiles/r6z*)
  const int wlog = ctx->stripe_log ? ctx->stripe_log : (K >= 16 ? 4 : K >= 8 ? 5 : 6), W = 1 << wlog;
  const long nstripes = (fx + W - 1) / W;
  const long capR = K > 1 ? 2L * fz * ((nstripes + K - 1) / K) + 64 : 0;
  const long ecells = K > 1 ? nstripes * 4L * fz : 0;  // per edge buffer (4 columns per stripe)
  // the band kernel's working field (af_band_tb_cells: its layout) and its edge buffers
  const long tb_cells = af_band_tb_cells(fz, fx), tbc = tb_cells + 2 * ecells, sbc = af_band_sb_cells(fz, fx);
  // the band kernel indexes the working field and both edge buffers with 32-bit cell indices
  if (tbc >= (1L << 31) - 1)
    return fail(ctx, ALIFMM_E_ARG, "travel: %d x %d grid with %ld edge cells exceeds the band kernel's 32-bit indexing",
                fz, fx, 2 * ecells);
  // the arena is sized for this chunk (reused while later chunks fit in it)
  int rc = ensure_arena(ctx, n, cells, sg > 1 ? cells : 0, capL, capC, capS, K, capR, ecells, tbc, sbc);
  if (rc) return rc;
  Arena& a = ctx->arena;
  // subgrid 1: the fields are first written by the band kernel, so their initialisation runs on
  // the fill stream beside the source-init kernel (which uses one CU per source); subgrid > 1:
  // the exact-stage kernel writes them, so in order on the main stream
  hipStream_t fs = (sg == 1 && ctx->fill) ? ctx->fill : ctx->stream;
  if (fs != ctx->stream) {  // the fill stream must not overwrite fields a previous call still reads
    HIPCHK(hipEventRecord(ctx->ev[3], ctx->stream));
    HIPCHK(hipStreamWaitEvent(fs, ctx->ev[3], 0));
  }
  std::vector<af::BandSrc> hs(n);
  for (int i = 0; i < n; i++) {
    int slot = first_slot + i;
    if ((rc = af_ensure_field(ctx, slot, sg, fz, fx))) return rc;
    af::BandSrc& b = hs[i];
    memset(&b, 0, sizeof b);
    b.T = ctx->fields[slot].d;
    b.S = sg > 1 ? a.S + (size_t)i * a.scells : nullptr;
    int* base = a.lists + (size_t)i * (4 * a.capL + 6 * a.capC);
    b.Lin = base;
    b.FS = base + a.capL;
    b.A = base + 2 * a.capL;
    b.L = base + 3 * a.capL;
    b.C = base + 4 * a.capL;
    b.Cp = b.C + a.capC;
    b.D = b.C + 2 * a.capC;
    b.Rx = b.C + 3 * a.capC;
    b.Bl = b.C + 4 * a.capC;
    b.Bp = b.C + 5 * a.capC;
    double* dbase = a.dlists + (size_t)i * (a.capL + 2 * a.capC);
    b.Lt = dbase;
    b.V = dbase + a.capL;
    b.Dv = b.V + a.capC;
    b.kx = a.kx + i;
    b.Tb = a.Tb + (size_t)i * a.tbc;
    HIPCHK(hipMemsetAsync(b.Tb, 0xFF, (size_t)tbc * 8, fs));  // far: NaN (working field + edge buffers)
    b.Sb = a.Sb + (size_t)i * a.sbc;
    HIPCHK(hipMemsetAsync(b.Sb, 0xFF, (size_t)sbc * 4, fs));  // kFar = -1
    if (K > 1) {
      b.rimc = a.rimc + (size_t)i * K * 2 * capR;
      b.rimt = a.rimt + (size_t)i * K * 2 * capR;
      b.E = b.Tb + tb_cells;  // edge buffers after the working field (fmm_band_k.hip indexes both from Tb)
    }
    if (capS > 0) {
      b.Ts[0] = a.Ts + (size_t)i * 2 * a.capS;
      b.Ts[1] = b.Ts[0] + a.capS;
      b.Ss[0] = a.Ss + (size_t)i * 2 * a.capS;
      b.Ss[1] = b.Ss[0] + a.capS;
    }
    // subgrid > 1: fmm_exact_kernel writes the exact region into the result field, which must
    // start far (NaN, fields.h); subgrid 1: the band kernel's copy-out writes every cell
    if (sg > 1) HIPCHK(hipMemsetAsync(b.T, 0xFF, (size_t)cells * 8, fs));
    if (sg > 1) HIPCHK(hipMemsetAsync(b.S, 0xFF, (size_t)cells * 4, fs));  // the exact kernel's status: kFar
  }
  if (fs != ctx->stream) HIPCHK(hipEventRecord(ctx->ev_fill, fs));
  HIPCHK(hipMemcpyAsync(a.srcs, hs.data(), sizeof(af::BandSrc) * n, hipMemcpyHostToDevice, ctx->stream));
  af::DevModel M = dev_model(ctx);
  af::BandParams P;
  memset(&P, 0, sizeof P);
  P.M = M;
  P.nsrc = n;
  P.sg = sg;
  P.nz = fz;
  P.nx = fx;
  P.dnx = ctx->dnx;
  P.dnz = ctx->dnz;
  P.cdelta = band_cdelta(ctx, sg);
  P.vmax = ctx->vmax;
  P.r0 = ctx->r0;
  P.cdelta_far = sg <= ctx->far_sg ? band_cdelta_far(ctx, sg) : 0.0;
  P.r_far = ctx->r_far;
  P.capL = (int)capL;
  P.capC = (int)capC;
  P.capS = (int)capS;
  P.src = a.srcs;
  P.gox = ctx->gox;
  P.goz = ctx->goz;
  P.prof = ctx->prof;
  P.coop = ctx->coop;
  P.K = K;
  P.wlog = wlog;
  P.capR = (int)capR;
  P.ecells = ecells;
  P.tb_pitch = af_band_tb_pitch(fx);
  P.tb_cells = tb_cells;
  P.sb_pitch = af_band_sb_pitch(fx);
  P.max_steps = 200L * (fz + fx) + 100000;
  if (so) {  // stream the fields to the host while the band runs (subgrid 1)
    so->active = false;
    if (sg == 1 && ctx->stream_out && (rc = stream_setup(ctx, so, n, K, wlog, fz, fx))) return rc;
    if (so->active) {
      P.hs = static_cast<double*>(ctx->hstage);
      P.hq = ctx->hq;
      P.hcons = ctx->hcons;
      P.qcap = so->g.qcap;
      P.rslots = so->g.rslots;
      P.tr_log = so->g.trlog;
    }
  }
  HIPCHK(hipEventRecord(ctx->ev[0], ctx->stream));
  if (sg == 1) {
    if (pre_ho) {  // initialised by the travel call for all its chunks (alifmm_travel)
      P.ho = const_cast<af::HandoverOut*>(pre_ho);
    } else {
      if ((rc = launch_source_init(ctx, n, scx, scz, a.jobs, a.ho))) return rc;
      P.ho = a.ho;
      ctx->ho_last = a.ho;
      ctx->n_ho_last = n;
    }
    P.mode = 0;
  } else {
    for (int i = 0; i < n; i++) {
      long ix = (long)std::nearbyint((scx[i] - ctx->gox) / ctx->dnx), iz = (long)std::nearbyint((scz[i] - ctx->goz) / ctx->dnz);
      if (ix < 0 || ix >= ctx->nx0 || iz < 0 || iz >= ctx->nz0)
        return fail(ctx, ALIFMM_E_ARG, "source %d (%g, %g) outside the grid", i, scx[i], scz[i]);
    }
    HIPCHK(hipMemcpyAsync(a.dscx, scx, 8 * n, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(a.dscz, scz, 8 * n, hipMemcpyHostToDevice, ctx->stream));
    P.mode = 1;
    P.scx = a.dscx;
    P.scz = a.dscz;
    // exact heap walk: both stage grids plus the fine-grid main loop out to exact_r fine nodes
    // beyond the stage-2 window (field units before the final / subgrid: coarse dnx per fine node)
    const long size2 = 2L * sg + (sg - 1) / 2 + 3L * sg;
    P.tstop = (double)(size2 + ctx->exact_r) * ctx->dnx / ctx->vmax;
    P.exact_r = ctx->exact_r;
    P.capL = (int)capL;
    P.capS = (int)capS;
    P.src = a.srcs;
    if (ctx->exact_lds && af_exact_lds_fits(sg, ctx->exact_r)) {
      HIPCHK(af_launch_exact_lds(&P, ctx->stream));
      // a heap past the LDS walk's capacity (error 9): those sources again, from scratch, with
      // the HBM walk (fmm_exact.hip)
      std::vector<af::BandSrc> chk(n);
      HIPCHK(hipMemcpyAsync(chk.data(), a.srcs, sizeof(af::BandSrc) * n, hipMemcpyDeviceToHost, ctx->stream));
      HIPCHK(hipStreamSynchronize(ctx->stream));
      bool redo = false;
      for (int i = 0; i < n; i++) redo |= chk[i].err == 9;
      for (int i = 0; i < n; i++) ctx->exact_redo += chk[i].err == 9;
      if (redo) {
        for (int i = 0; i < n; i++) {
          HIPCHK(hipMemsetAsync(hs[i].T, 0xFF, (size_t)cells * 8, ctx->stream));
          HIPCHK(hipMemsetAsync(hs[i].S, 0xFF, (size_t)cells * 4, ctx->stream));
        }
        HIPCHK(hipMemcpyAsync(a.srcs, hs.data(), sizeof(af::BandSrc) * n, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(af_launch_exact(&P, ctx->stream));
      }
    } else {
      HIPCHK(af_launch_exact(&P, ctx->stream));
    }
  }
  HIPCHK(hipEventRecord(ctx->ev[1], ctx->stream));
  if (fs != ctx->stream) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_fill, 0));
  HIPCHK(hipMemsetAsync(a.kx, 0, sizeof(af::KX) * n, ctx->stream));
  HIPCHK(af_launch_band_k(&P, ctx->stream));
  // the copy team takes the tiles as they arrive; joined on every return path below
  struct StreamJoin {
    alifmm_ctx* c;
    StreamOut* s;
    ~StreamJoin() {
      if (!s) return;
      // an early return: the kernel may still store into the pinned ring; it must have ended
      // before the drain stops and the next call resets or frees those buffers
      (void)hipStreamSynchronize(c->stream);
      (void)hipGetLastError();
      stream_finish(c, s);
    }
  } sjoin{ctx, nullptr};
  if (so && so->active) {
    stream_start(ctx, so);
    sjoin.s = so;
  }
  ctx->last_k = K;
  HIPCHK(hipEventRecord(ctx->ev[2], ctx->stream));
  if (sg > 1)
    for (int i = 0; i < n; i++) HIPCHK(af_launch_scale(hs[i].T, cells, (double)sg, ctx->stream));
  HIPCHK(hipMemcpyAsync(hs.data(), a.srcs, sizeof(af::BandSrc) * n, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (sjoin.s) {
    stream_finish(ctx, so);
    sjoin.s = nullptr;
  }
  float t1 = 0, t2 = 0;
  (void)hipEventElapsedTime(&t1, ctx->ev[0], ctx->ev[1]);
  (void)hipEventElapsedTime(&t2, ctx->ev[1], ctx->ev[2]);
  *ms_init += t1;
  *ms_band += t2;
  int cap_err = 0;
  for (int i = 0; i < n; i++) {
    Field& f = ctx->fields[first_slot + i];
    for (int k = 0; k < 4; k++) f.steps[k] = hs[i].steps[k];
    f.sweeps = hs[i].nupd;
    for (int k = 0; k < 6; k++) f.prof[k] = hs[i].ph[k];
    for (int k = 0; k < 3; k++) f.prof[6 + k] = hs[i].lsum[k];
    f.prof[9] = hs[i].lmax;
    f.span[0] = hs[i].t_begin;
    f.span[1] = hs[i].t_end;
    for (int k = 0; k < 4; k++) f.prof[10 + k] = hs[i].sub[k];
    if (hs[i].err == 2) cap_err = 1;
    else if (hs[i].err == 3) return fail(ctx, ALIFMM_E_KERNEL, "source %d: init heap overflow", i);
    else if (hs[i].err == 4) return fail(ctx, ALIFMM_E_KERNEL, "source %d: stage grid capacity", i);
    else if (hs[i].err == 7 && !P.coop) return fail(ctx, kRetryCoop, "source %d: band members not co-resident", i);
    else if (hs[i].err) return fail(ctx, ALIFMM_E_KERNEL, "source %d: kernel error %d", i, hs[i].err);
  }
  if (cap_err) return fail(ctx, ALIFMM_E_CAPACITY, "work-list capacity %ld exceeded", capL);
  return ALIFMM_OK;
}

// dsts: per source, the caller's (pageable) field, or null (the fields stay resident only)
static int travel_impl(alifmm_ctx* ctx, int subgrid, int nsrc, const double* scx, const double* scz, int first_slot,
                       double* const* dsts) {
  if (!ctx || !ctx->have_model) return fail(ctx, ALIFMM_E_ARG, "travel: no model");
  if ((long)subgrid * (ctx->nz0 - 1) + 1 >= 32768 || (long)subgrid * (ctx->nx0 - 1) + 1 >= 32768)
    return fail(ctx, ALIFMM_E_ARG, "travel: field sides must stay below 32768 nodes (packed list keys)");
  if (subgrid < 1 || subgrid % 2 == 0) return fail(ctx, ALIFMM_E_ARG, "travel: subgrid must be odd, got %d", subgrid);
  if (nsrc < 0 || first_slot < 0 || (nsrc > 0 && (!scx || !scz))) return fail(ctx, ALIFMM_E_ARG, "travel: bad args");
  HIPCHK(hipSetDevice(ctx->device));
  int fz, fx;
  alifmm_field_shape(ctx, subgrid, &fz, &fx);
  const long cells = (long)fz * fx;
  float ms_init = 0, ms_band = 0;
  // Sources per launch: at most half the CUs, so that every source gets >= 2 band members (256
  // C5 receivers on 256 CUs: one launch with one member each 927 ms, two launches of 128 with two
  // members each 810 ms, profiles/r3w_batch.json), balanced over the launches (multiples of 8)
  int chunk = std::max(1, std::min(ctx->batch, std::max(8, ctx->n_cu / 2 / 8 * 8)));
  if (nsrc > chunk) {
    const int nl = (nsrc + chunk - 1) / chunk;
    chunk = std::min(chunk, ((nsrc + nl - 1) / nl + 7) / 8 * 8);
  }
  // subgrid 1 over several launches: one source-init launch for every source of the call (the
  // init uses one CU per source; chunk by chunk it would run alone before each band launch)
  const bool pre_init = subgrid == 1 && nsrc > chunk;
  if (pre_init && ctx->n_all < nsrc) {
    if (ctx->ho_last == ctx->ho_all) {
      ctx->ho_last = nullptr;
      ctx->n_ho_last = 0;
    }
    dfree(ctx->ho_all);
    dfree(ctx->jobs_all);
    ctx->ho_all = nullptr;
    ctx->jobs_all = nullptr;
    ctx->n_all = 0;
    HIPCHK(dalloc(&ctx->ho_all, nsrc));
    HIPCHK(dalloc(&ctx->jobs_all, nsrc));
    ctx->n_all = nsrc;
  }
  ctx->t_stream_tail = 0;
  ctx->stream_fallback = 0;
  ctx->exact_redo = 0;
  HIPCHK(hipEventRecord(ctx->ev[3], ctx->stream));
  // the call's timing events, destroyed on every return path
  struct Ev {
    hipEvent_t e = nullptr;
    ~Ev() {
      if (e) (void)hipEventDestroy(e);
    }
  } t_begin, t_end;
  HIPCHK(hipEventCreate(&t_begin.e));
  HIPCHK(hipEventCreate(&t_end.e));
  HIPCHK(hipEventRecord(t_begin.e, ctx->stream));
  const af::HandoverOut* pre = nullptr;
  if (pre_init) {
    HIPCHK(hipEventRecord(ctx->ev[0], ctx->stream));
    int rc = launch_source_init(ctx, nsrc, scx, scz, ctx->jobs_all, ctx->ho_all);
    if (rc) return rc;
    HIPCHK(hipEventRecord(ctx->ev[1], ctx->stream));
    HIPCHK(hipEventSynchronize(ctx->ev[1]));
    float t = 0;
    (void)hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[1]);
    ms_init += t;
    pre = ctx->ho_all;
    ctx->ho_last = ctx->ho_all;
    ctx->n_ho_last = nsrc;
  }
  for (int s0 = 0; s0 < nsrc; s0 += chunk) {
    int n = std::min(chunk, nsrc - s0);
    int rc;
    StreamOut so;
    so.dst = dsts ? dsts + s0 : nullptr;
    so.n = n;
    StreamOut* sop = dsts ? &so : nullptr;
    for (;;) {
      rc = travel_chunk(ctx, subgrid, n, scx + s0, scz + s0, first_slot + s0, fz, fx, &ms_init, &ms_band,
                        pre ? pre + s0 : nullptr, sop);
      if (rc == kRetryCoop) {  // once, gang-scheduled
        const int c0 = ctx->coop;
        ctx->coop = 1;
        rc = travel_chunk(ctx, subgrid, n, scx + s0, scz + s0, first_slot + s0, fz, fx, &ms_init, &ms_band,
                          pre ? pre + s0 : nullptr, sop);
        ctx->coop = c0;
        if (rc == kRetryCoop) rc = ALIFMM_E_KERNEL;
      }
      if (rc != ALIFMM_E_CAPACITY || ctx->cap_scale * 4 > 64) break;
      ctx->cap_scale *= 4;  // retry the chunk with larger work lists
    }
    if (rc) return rc;
    if (dsts) {  // fields not streamed (or a tile that never arrived): through the pinned staging ring
      for (int i = 0; i < n; i++) {
        if (so.active && !so.missing[i].load()) continue;
        if (so.active) ctx->stream_fallback++;
        rc = alifmm_copy_fields(ctx, first_slot + s0 + i, 1, dsts[s0 + i], 0, nullptr);
        if (rc) return rc;
      }
    }
  }
  HIPCHK(hipEventRecord(t_end.e, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  float tot = 0;
  (void)hipEventElapsedTime(&tot, t_begin.e, t_end.e);
  ctx->t_init = ms_init;
  ctx->t_band = ms_band;
  ctx->t_total = tot;
  return ALIFMM_OK;
}

int alifmm_travel(alifmm_ctx* ctx, int subgrid, int nsrc, const double* scx, const double* scz, int first_slot,
                  double* out) {
  if (!out) return travel_impl(ctx, subgrid, nsrc, scx, scz, first_slot, nullptr);
  int fz = 0, fx = 0;
  if (ctx && ctx->have_model) alifmm_field_shape(ctx, subgrid, &fz, &fx);
  std::vector<double*> d(std::max(nsrc, 0));
  for (int i = 0; i < nsrc; i++) d[i] = out + (size_t)i * fz * fx;
  return travel_impl(ctx, subgrid, nsrc, scx, scz, first_slot, d.data());
}

int alifmm_travel_into(alifmm_ctx* ctx, int subgrid, int nsrc, const double* scx, const double* scz, int first_slot,
                       double* const* dst) {
  if (nsrc > 0 && !dst) return fail(ctx, ALIFMM_E_ARG, "travel_into: no destinations");
  for (int i = 0; i < nsrc; i++)
    if (!dst[i]) return fail(ctx, ALIFMM_E_ARG, "travel_into: destination %d is null", i);
  return travel_impl(ctx, subgrid, nsrc, scx, scz, first_slot, dst);
}

int alifmm_get_field(alifmm_ctx* ctx, int slot, double* out) {
  if (!ctx || slot < 0 || slot >= (int)ctx->fields.size() || !ctx->fields[slot].d || !out)
    return fail(ctx, ALIFMM_E_ARG, "get_field: no field in slot %d", slot);
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMemcpyAsync(out, ctx->fields[slot].d, ctx->fields[slot].bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return ALIFMM_OK;
}

// Host copy of one staged piece by a persistent team of threads (one slice each), one team per
// context (created on first use, joined by alifmm_ctx_destroy); its size is OMP_NUM_THREADS when
// set (the job's CPU share on the GPU box, 16), else up to 8.  Creating the threads per piece cost
// ~0.1 ms per 32 MiB piece (≈60 ms for a 17 GB stack).
class CopyTeam {
 public:
  explicit CopyTeam(int n) : n_(n) {
    for (int t = 1; t < n_; t++) th_.emplace_back([this, t] { run(t); });
  }
  ~CopyTeam() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return n_; }
  // f(t) on the team's threads t = 1 .. size() - 1 (not the caller's); wait() joins them
  void start(std::function<void(int)> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = std::move(f);
      left_ = n_ - 1;
      gen_++;
    }
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> l(m_);
    done_.wait(l, [&] { return left_ == 0; });
  }
  void copy(char* dst, const char* src, size_t n) {
    if (n_ <= 1 || n < (4u << 20)) {
      memcpy(dst, src, n);
      return;
    }
    dst_ = dst;
    src_ = src;
    bytes_ = n;
    start([this](int t) { slice(t); });
    slice(0);
    wait();
  }

 private:
  void slice(int t) const {
    const size_t s = ((bytes_ + n_ - 1) / n_ + 4095) & ~(size_t)4095, o = (size_t)t * s;
    if (o < bytes_) memcpy(dst_ + o, src_ + o, std::min(s, bytes_ - o));
  }
  void run(int t) {
    unsigned long seen = 0;
    for (;;) {
      std::function<void(int)> f;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        f = job_;
      }
      f(t);
      std::lock_guard<std::mutex> g(m_);
      if (--left_ == 0) done_.notify_one();
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  std::function<void(int)> job_;
  char* dst_ = nullptr;
  const char* src_ = nullptr;
  size_t bytes_ = 0;
  int left_ = 0;
  unsigned long gen_ = 0;
  bool stop_ = false;
};

static CopyTeam& copy_team(alifmm_ctx* ctx) {
  if (!ctx->team) {
    // the process's CPU share (OMP_NUM_THREADS on the GPU box, else up to 8) split over the live
    // contexts (one per GPU in update_parallel), at least two threads per team (caller + one)
    int n = (int)std::min(8u, std::max(1u, std::thread::hardware_concurrency()));
    if (const char* e = getenv("OMP_NUM_THREADS")) {
      const int v = atoi(e);
      if (v >= 1) n = std::min(v, 32);
    }
    n = std::max(2, n / std::max(1, g_live_ctx.load()));
    ctx->team = new CopyTeam(n);
  }
  return *static_cast<CopyTeam*>(ctx->team);
}
static void destroy_team(alifmm_ctx* ctx) {
  delete static_cast<CopyTeam*>(ctx->team);
  ctx->team = nullptr;
}

static void free_stream_bufs(alifmm_ctx* ctx) {
  if (ctx->hstage) (void)hipHostFree(ctx->hstage);
  if (ctx->hq) (void)hipHostFree(ctx->hq);
  if (ctx->hcons) (void)hipHostFree(ctx->hcons);
  ctx->hstage = nullptr;
  ctx->hq = nullptr;
  ctx->hcons = nullptr;
  ctx->hstage_bytes = ctx->hq_bytes = ctx->hcons_bytes = 0;
}

static int host_buf(void** p, size_t* have, size_t need) {  // coherent pinned memory, grown on demand
  if (*have >= need) return 0;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *have = 0;
  if (hipHostMalloc(p, need, hipHostMallocCoherent) != hipSuccess) {
    (void)hipGetLastError();
    *p = nullptr;
    return -1;
  }
  *have = need;
  return 0;
}

// Tile geometry (tile_stream.h) and host buffers of a streamed band launch: a ring of
// kRingSlots tile slots per member (1 GB at C4).  No geometry, no copy team or no pinned memory:
// so->active stays false (the fields are copied after the launch).
static int stream_setup(alifmm_ctx* ctx, StreamOut* so, int n, int K, int wlog, int fz, int fx) {
  so->active = false;
  if (copy_team(ctx).size() < 2 || !af::ts::plan(K, wlog, fz, fx, &so->g)) return ALIFMM_OK;
  const af::ts::Geometry& g = so->g;
  const size_t members = (size_t)n * K, tile_bytes = ((size_t)1 << g.clog()) * sizeof(double);
  const size_t qbytes = members * g.qcap * sizeof(unsigned long long);
  if (host_buf(&ctx->hstage, &ctx->hstage_bytes, members * g.rslots * tile_bytes) ||
      host_buf((void**)&ctx->hq, &ctx->hq_bytes, qbytes) ||
      host_buf((void**)&ctx->hcons, &ctx->hcons_bytes, members * sizeof(unsigned))) {
    free_stream_bufs(ctx);
    return ALIFMM_OK;
  }
  // (the previous launch that used them has completed)
  memset(ctx->hq, 0, qbytes);
  memset(ctx->hcons, 0, members * sizeof(unsigned));
  so->active = true;
  return ALIFMM_OK;
}

static void stream_start(alifmm_ctx* ctx, StreamOut* so) {
  CopyTeam& team = copy_team(ctx);
  so->kernel_done.store(0);
  so->missing.reset(new std::atomic<int>[so->n]);
  for (int i = 0; i < so->n; i++) so->missing[i].store(0);
  const int nw = team.size() - 1;
  const af::ts::Buffers b{static_cast<const double*>(ctx->hstage), ctx->hq, ctx->hcons};
  team.start([so, b, nw](int t) {
    af::ts::drain(so->g, so->n, so->dst, b, t - 1, nw,
                  [so] { return so->kernel_done.load(std::memory_order_acquire) != 0; }, so->missing.get());
  });
}

// the launch has completed (or failed): the workers finish the queues, then the team is joined
static void stream_finish(alifmm_ctx* ctx, StreamOut* so) {
  const auto t0 = std::chrono::steady_clock::now();
  so->kernel_done.store(1, std::memory_order_release);
  copy_team(ctx).wait();
  ctx->t_stream_tail += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// Device -> pageable host copy of a list of segments: pieces of kPinBytes through kPinBufs pinned
// buffers; the DMA of the next pieces runs while a thread team copies the current one out of its
// buffer (alifmm_copy_fields, alifmm_take_rays)
struct D2HSeg {
  const char* src;
  char* dst;
  size_t bytes;
};
static int d2h_pageable(alifmm_ctx* ctx, const std::vector<D2HSeg>& segs) {
  const int nb = alifmm_ctx::kPinBufs;
  const size_t pb = alifmm_ctx::kPinBytes;
  size_t total = 0;
  for (const auto& g : segs) total += g.bytes;
  if (total <= kSmallD2H && !ctx->pin[0]) {
    // a small copy before the ring exists (e.g. the weld example's 8 MB of ray points): plain copies,
    // not 4 x 32 MB of fresh pinned memory (~30 ms to allocate) and a copy team
    for (const auto& g : segs) HIPCHK(hipMemcpyAsync(g.dst, g.src, g.bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return ALIFMM_OK;
  }
  for (int b = 0; b < nb; b++) {
    if (!ctx->pin[b]) HIPCHK(hipHostMalloc(&ctx->pin[b], pb, hipHostMallocDefault));
    if (!ctx->pin_ev[b]) HIPCHK(hipEventCreateWithFlags(&ctx->pin_ev[b], hipEventDisableTiming));
  }
  std::vector<D2HSeg> pieces;
  for (const auto& g : segs)
    for (size_t o = 0; o < g.bytes; o += pb) pieces.push_back({g.src + o, g.dst + o, std::min(pb, g.bytes - o)});
  const long np = (long)pieces.size();
  auto issue = [&](long i) -> hipError_t {
    hipError_t e = hipMemcpyAsync(ctx->pin[i % nb], pieces[i].src, pieces[i].bytes, hipMemcpyDeviceToHost, ctx->stream);
    return e == hipSuccess ? hipEventRecord(ctx->pin_ev[i % nb], ctx->stream) : e;
  };
  CopyTeam& team = copy_team(ctx);
  for (long i = 0; i < std::min<long>(nb, np); i++) HIPCHK(issue(i));
  for (long i = 0; i < np; i++) {
    HIPCHK(hipEventSynchronize(ctx->pin_ev[i % nb]));
    team.copy(pieces[i].dst, (const char*)ctx->pin[i % nb], pieces[i].bytes);
    if (i + nb < np) HIPCHK(issue(i + nb));
  }
  return ALIFMM_OK;
}

int alifmm_copy_fields(alifmm_ctx* ctx, int first_slot, int n, double* dst, int dst_kind, double* gbps) {
  if (!ctx || n < 0 || first_slot < 0 || (n > 0 && !dst) || dst_kind < 0 || dst_kind > 3)
    return fail(ctx, ALIFMM_E_ARG, "copy_fields: bad args");
  if (n == 0) return ALIFMM_OK;
  if (first_slot + n > (int)ctx->fields.size()) return fail(ctx, ALIFMM_E_ARG, "copy_fields: slots out of range");
  const size_t fb = ctx->fields[first_slot].bytes;
  for (int i = 0; i < n; i++)
    if (!ctx->fields[first_slot + i].d || ctx->fields[first_slot + i].bytes != fb)
      return fail(ctx, ALIFMM_E_ARG, "copy_fields: slot %d empty or of another shape", first_slot + i);
  HIPCHK(hipSetDevice(ctx->device));
  const auto t0 = std::chrono::steady_clock::now();
  char* out = (char*)dst;
  bool registered = false;
  if (dst_kind == 3) {  // pageable destination registered for this copy: the DMA writes it directly
    HIPCHK(hipHostRegister(dst, (size_t)n * fb, hipHostRegisterDefault));
    registered = true;
    dst_kind = 1;
  }
  if (dst_kind != 0) {  // one DMA per field (device -> device, or into host memory the DMA can write)
    const hipMemcpyKind kind = dst_kind == 2 ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    hipError_t e = hipSuccess;
    for (int i = 0; i < n && e == hipSuccess; i++)
      e = hipMemcpyAsync(out + (size_t)i * fb, ctx->fields[first_slot + i].d, fb, kind, ctx->stream);
    const hipError_t es = hipStreamSynchronize(ctx->stream);
    if (registered) (void)hipHostUnregister(dst);
    if (e != hipSuccess || es != hipSuccess)
      return fail(ctx, ALIFMM_E_HIP, "copy_fields: %s", hipGetErrorString(e != hipSuccess ? e : es));
  } else {
    std::vector<D2HSeg> segs(n);
    for (int i = 0; i < n; i++) segs[i] = {(const char*)ctx->fields[first_slot + i].d, out + (size_t)i * fb, fb};
    const int rc = d2h_pageable(ctx, segs);
    if (rc) return rc;
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (gbps) *gbps = dt > 0 ? (double)fb * n / dt / 1e9 : 0.0;
  return ALIFMM_OK;
}

int alifmm_source_stats(alifmm_ctx* ctx, int slot, int64_t* steps4, int64_t* cell_sweeps) {
  if (!ctx || slot < 0 || slot >= (int)ctx->fields.size()) return fail(ctx, ALIFMM_E_ARG, "stats: bad slot");
  if (steps4)
    for (int k = 0; k < 4; k++) steps4[k] = ctx->fields[slot].steps[k];
  if (cell_sweeps) *cell_sweeps = ctx->fields[slot].sweeps;
  return ALIFMM_OK;
}

int alifmm_band_profile(alifmm_ctx* ctx, int slot, int64_t* out14) {
  if (!ctx || slot < 0 || slot >= (int)ctx->fields.size() || !out14) return fail(ctx, ALIFMM_E_ARG, "band_profile: bad slot");
  for (int k = 0; k < 14; k++) out14[k] = ctx->fields[slot].prof[k];
  return ALIFMM_OK;
}

int alifmm_band_span(alifmm_ctx* ctx, int slot, int64_t* out2) {
  if (!ctx || slot < 0 || slot >= (int)ctx->fields.size() || !out2) return fail(ctx, ALIFMM_E_ARG, "band_span: bad slot");
  out2[0] = ctx->fields[slot].span[0];
  out2[1] = ctx->fields[slot].span[1];
  return ALIFMM_OK;
}

int alifmm_init_profile(alifmm_ctx* ctx, int i, int64_t* out16) {
  if (!ctx || !out16 || i < 0 || i >= ctx->n_ho_last || !ctx->ho_last)
    return fail(ctx, ALIFMM_E_ARG, "init_profile: bad index");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMemcpy(out16, &ctx->ho_last[i].prof[0], 16 * sizeof(long long), hipMemcpyDeviceToHost));
  return ALIFMM_OK;
}

int alifmm_last_timing(alifmm_ctx* ctx, double* init_ms, double* band_ms, double* total_ms) {
  if (!ctx) return ALIFMM_E_ARG;
  if (init_ms) *init_ms = ctx->t_init;
  if (band_ms) *band_ms = ctx->t_band;
  if (total_ms) *total_ms = ctx->t_total;
  return ALIFMM_OK;
}

int alifmm_find_rays(alifmm_ctx* ctx, int npairs, const int32_t* field_slot, const double* src_xy,
                     const double* rec_xy, double* times, int32_t* ray_len, int32_t* flags, double* ray_xy,
                     int64_t ray_xy_cap) {
  if (!ctx || !ctx->have_model) return fail(ctx, ALIFMM_E_ARG, "find_rays: no model");
  if (npairs <= 0) return ALIFMM_OK;
  HIPCHK(hipSetDevice(ctx->device));
  const auto t_call = std::chrono::steady_clock::now();
  ctx->t_ray_kernel = ctx->t_ray_pack = 0;
  const int max_pts = 5 * (ctx->nz0 + ctx->nx0);
  // group rays by subgrid (one launch per subgrid size present)
  std::map<int, std::vector<int>> by_sg;
  for (int k = 0; k < npairs; k++) {
    int s = field_slot[k];
    if (s < 0 || s >= (int)ctx->fields.size() || !ctx->fields[s].d)
      return fail(ctx, ALIFMM_E_ARG, "find_rays: ray %d refers to empty slot %d", k, s);
    by_sg[ctx->fields[s].sg].push_back(k);
  }
  for (auto& g : by_sg)
    if (6 * g.first + 3 > kMaxRayCand)  // the plane search keeps <= kMaxRayCand candidates per ray (rays.hip)
      return fail(ctx, ALIFMM_E_ARG, "find_rays: subgrid %d has %d plane candidates (> %d supported)", g.first,
                  6 * g.first + 3, kMaxRayCand);
  // chunk of rays per launch; the point buffers (chunk x max_pts per coordinate) are sized to the
  // request and kept in the context for the next call
  // Rays per launch: wavefronts for every SIMD at the ray kernel's occupancy (af_ray_waves_per_simd;
  // 8 192 rays at 16 lanes per ray and 2 wavefronts per SIMD), balanced over the launches, with the
  // point buffers within a quarter of the free device memory.
  int chunk = 8192;
  int ray_packed = 0;
  size_t keep_budget = SIZE_MAX;  // device bytes the kept points of this call may hold (a quarter of the free memory)
  {
    // 9-lane groups (7 rays per wavefront) only for requests that fill the device with them: fewer
    // rays in 16-lane groups give every SIMD its wavefronts (8 192 rays: 0.130 s vs 0.173 s,
    // profiles/r5e)
    const long fill9 = (long)std::max(ctx->n_cu, 1) * 4 * af_ray_waves_per_simd() * (64 / 9);
    ray_packed = npairs >= fill9 ? 1 : 0;
    int rays_per_wave = 64;
    for (auto& g : by_sg) rays_per_wave = std::min(rays_per_wave, 64 / af_ray_group_lanes(g.first, ray_packed));
    const long target = (long)std::max(ctx->n_cu, 1) * 4 * af_ray_waves_per_simd() * rays_per_wave;
    size_t free_b = 0, total_b = 0;
    long by_mem = target;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
      by_mem = (long)(free_b / 4 / ((size_t)max_pts * 2 * sizeof(double) + 64));
      keep_budget = free_b / 4;
    }
    const long cmax = std::max(1024L, std::min(target, by_mem));
    const long nlaunch = (npairs + cmax - 1) / cmax;
    chunk = (int)((npairs + nlaunch - 1) / nlaunch);
  }
  chunk = std::min(chunk, npairs);
  auto& rb = ctx->rb;
  if (rb.rays < chunk || rb.pts < (size_t)chunk * max_pts) {
    free_ray_bufs(ctx);
    HIPCHK(dalloc(&rb.rx, (size_t)chunk * max_pts));
    HIPCHK(dalloc(&rb.ry, (size_t)chunk * max_pts));
    HIPCHK(dalloc(&rb.t, chunk));
    HIPCHK(dalloc(&rb.len, chunk));
    HIPCHK(dalloc(&rb.flags, chunk));
    HIPCHK(dalloc(&rb.jobs, chunk));
    HIPCHK(dalloc(&rb.off, chunk));
    rb.rays = chunk;
    rb.pts = (size_t)chunk * max_pts;
  }
  double *d_rx = rb.rx, *d_ry = rb.ry, *d_t = rb.t, *d_packed = nullptr;
  int *d_len = rb.len, *d_flags = rb.flags;
  af::RayJob* d_jobs = rb.jobs;
  long long* d_off = rb.off;
  int rc = ALIFMM_OK;
  auto cleanup = [&]() { dfree(d_packed); };
  // an error return also drops the points kept so far (kept_pts then matches no ray list)
#define RCHK(call)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess) {                                                               \
      cleanup();                                                                          \
      release_kept_rays(ctx);                                                             \
      return fail(ctx, ALIFMM_E_HIP, "%s: %s", #call, hipGetErrorString(e_));             \
    }                                                                                     \
  } while (0)
  std::vector<int64_t> offsets(npairs + 1, 0);
  std::vector<int32_t> lens(npairs, 0);
  std::vector<double> tms(npairs, 0.0);
  std::vector<int32_t> flg(npairs, 0);
  // pass 1: trace, lengths
  struct Pending { std::vector<int> ids; };
  std::vector<std::pair<int, std::vector<int>>> groups(by_sg.begin(), by_sg.end());
  // Rays are traced chunk by chunk; packed points are written after lengths are known (pass 2 re-traces
  // nothing: each chunk is packed right after its trace, at offsets relative to the ray order below).
  std::vector<int> order;
  for (auto& g : groups) order.insert(order.end(), g.second.begin(), g.second.end());
  // offsets follow the caller's ray order; we first trace everything (times/lengths), packing each
  // chunk into a host staging area keyed by ray id.
  const bool keep = !ray_xy && ray_xy_cap == ALIFMM_KEEP_RAYS;
  // one subgrid (the usual case): the rays are traced in the caller's order, so the kept points
  // stay on the device, chunk after chunk, and alifmm_take_rays copies them out once
  // (while the kept bytes stay within keep_budget; past it the kept chunks move to host staging)
  bool dev_keep = keep && groups.size() == 1;
  release_kept_rays(ctx);
  std::vector<std::vector<double>> staged(((ray_xy || keep) && !dev_keep) ? npairs : 0);
  size_t kept_bytes = 0;
  // device-kept chunks -> per-ray host staging (rays ids[0 .. ndone-1] of the single group, in order)
  auto spill_kept = [&](const std::vector<int>& ids) -> hipError_t {
    staged.assign(npairs, {});
    size_t r = 0;
    for (auto& k : ctx->kept_dev) {
      std::vector<double> h(2 * (size_t)k.npts);
      hipError_t e = hipMemcpy(h.data(), k.d, 16 * (size_t)k.npts, hipMemcpyDeviceToHost);
      if (e != hipSuccess) return e;
      size_t o = 0;
      while (o < (size_t)k.npts) {
        const int id = ids[r++];
        staged[id].assign(h.begin() + 2 * o, h.begin() + 2 * (o + lens[id]));
        o += lens[id];
      }
    }
    for (auto& k : ctx->kept_dev) dfree(k.d);
    ctx->kept_dev.clear();
    ctx->kept_pts = 0;
    dev_keep = false;
    return hipSuccess;
  };
  for (auto& g : groups) {
    const int sg = g.first;
    const auto& ids = g.second;
    const Field& f0 = ctx->fields[field_slot[ids[0]]];
    for (size_t c0 = 0; c0 < ids.size(); c0 += chunk) {
      int n = (int)std::min<size_t>(chunk, ids.size() - c0);
      std::vector<af::RayJob> jobs(n);
      for (int i = 0; i < n; i++) {
        int k = ids[c0 + i];
        const Field& f = ctx->fields[field_slot[k]];
        jobs[i].ttf = f.d;
        jobs[i].sx = src_xy[2 * k];
        jobs[i].sy = src_xy[2 * k + 1];
        jobs[i].rx = rec_xy[2 * k];
        jobs[i].ry = rec_xy[2 * k + 1];
        if (f.nz != f0.nz || f.nx != f0.nx) {
          cleanup();
          release_kept_rays(ctx);
          return fail(ctx, ALIFMM_E_ARG, "find_rays: mixed field shapes for subgrid %d", sg);
        }
      }
      RCHK(hipMemcpyAsync(d_jobs, jobs.data(), sizeof(af::RayJob) * n, hipMemcpyHostToDevice, ctx->stream));
      af::RayParams P;
      memset(&P, 0, sizeof P);
      P.M = dev_model(ctx);
      P.fnz = f0.nz;
      P.fnx = f0.nx;
      P.sg = sg;
      P.dnx = ctx->dnx;
      P.nrays = n;
      P.max_pts = max_pts;
      P.jobs = d_jobs;
      P.ray_x = d_rx;
      P.ray_y = d_ry;
      P.ray_len = d_len;
      P.times = d_t;
      P.flags = d_flags;
      P.glanes = af_ray_group_lanes(sg, ray_packed);
      ctx->last_ray_lanes = P.glanes;
      RCHK(hipEventRecord(ctx->ev[0], ctx->stream));
      RCHK(af_launch_rays(&P, ctx->stream));
      RCHK(hipEventRecord(ctx->ev[1], ctx->stream));
      std::vector<double> t(n);
      std::vector<int> l(n), fl(n);
      RCHK(hipMemcpyAsync(t.data(), d_t, 8 * n, hipMemcpyDeviceToHost, ctx->stream));
      RCHK(hipMemcpyAsync(l.data(), d_len, 4 * n, hipMemcpyDeviceToHost, ctx->stream));
      RCHK(hipMemcpyAsync(fl.data(), d_flags, 4 * n, hipMemcpyDeviceToHost, ctx->stream));
      RCHK(hipStreamSynchronize(ctx->stream));
      {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]);
        ctx->t_ray_kernel += ms;
      }
      for (int i = 0; i < n; i++) {
        int k = ids[c0 + i];
        tms[k] = t[i];
        lens[k] = l[i];
        flg[k] = fl[i];
      }
      if (ray_xy || keep) {
        std::vector<long long> off(n + 1, 0);
        for (int i = 0; i < n; i++) off[i + 1] = off[i] + l[i];
        dfree(d_packed);
        d_packed = nullptr;
        RCHK(dalloc(&d_packed, (size_t)2 * std::max<long long>(off[n], 1)));
        RCHK(hipMemcpyAsync(d_off, off.data(), 8 * n, hipMemcpyHostToDevice, ctx->stream));
        RCHK(hipEventRecord(ctx->ev[2], ctx->stream));
        RCHK(af_launch_pack_rays(d_rx, d_ry, d_len, d_off, n, max_pts, d_packed, ctx->stream));
        RCHK(hipEventRecord(ctx->ev[3], ctx->stream));
        RCHK(hipEventSynchronize(ctx->ev[3]));
        {
          float ms = 0;
          (void)hipEventElapsedTime(&ms, ctx->ev[2], ctx->ev[3]);
          ctx->t_ray_pack += ms;
        }
        if (dev_keep && kept_bytes + 16 * (size_t)off[n] > keep_budget) RCHK(spill_kept(ids));
        if (dev_keep) {  // the chunk's packed points stay on the device (the context owns them now)
          kept_bytes += 16 * (size_t)off[n];
          ctx->kept_dev.push_back({d_packed, (int64_t)off[n]});
          ctx->kept_pts += off[n];
          d_packed = nullptr;
          continue;
        }
        std::vector<double> packed(2 * off[n]);
        RCHK(hipMemcpyAsync(packed.data(), d_packed, 16 * off[n], hipMemcpyDeviceToHost, ctx->stream));
        RCHK(hipStreamSynchronize(ctx->stream));
        for (int i = 0; i < n; i++)
          staged[ids[c0 + i]].assign(packed.begin() + 2 * off[i], packed.begin() + 2 * off[i + 1]);
      }
    }
  }
  for (int k = 0; k < npairs; k++) offsets[k + 1] = offsets[k] + lens[k];
  if (ray_xy && offsets[npairs] > ray_xy_cap) rc = fail(ctx, ALIFMM_E_ARG, "find_rays: ray_xy capacity %lld < %lld",
                                                      (long long)ray_xy_cap, (long long)offsets[npairs]);
  if (!rc) {
    for (int k = 0; k < npairs; k++) {
      times[k] = tms[k];
      ray_len[k] = lens[k];
      if (flags) flags[k] = flg[k];
      if (ray_xy) std::copy(staged[k].begin(), staged[k].end(), ray_xy + 2 * offsets[k]);
    }
    if (keep && !dev_keep) {
      ctx->kept_rays.swap(staged);
      ctx->kept_pts = offsets[npairs];
    }
  }
  if (rc || (dev_keep && ctx->kept_pts != offsets[npairs])) {
    release_kept_rays(ctx);
    if (!rc) rc = fail(ctx, ALIFMM_E_KERNEL, "find_rays: kept points do not add up to the ray lengths");
  }
  cleanup();
  ctx->t_find_rays = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count();
  // point buffers above kRayBufKeepBytes (C4: 8192 rays x 40 960 points x 16 B = 5.4 GB) are not kept
  // between calls, so they do not hold device memory that later travel / arena allocations need
  if (rb.pts * 2 * sizeof(double) > kRayBufKeepBytes) free_ray_bufs(ctx);
  return rc;
}

int alifmm_take_rays(alifmm_ctx* ctx, double* ray_xy, int64_t ray_xy_cap, int64_t* n_points) {
  if (!ctx) return ALIFMM_E_ARG;
  if (n_points) *n_points = ctx->kept_pts;
  if (!ray_xy) return ALIFMM_OK;  // size query
  if (ray_xy_cap < ctx->kept_pts)
    return fail(ctx, ALIFMM_E_ARG, "take_rays: ray_xy capacity %lld < %lld", (long long)ray_xy_cap,
                (long long)ctx->kept_pts);
  int64_t off = 0;
  const auto t_call = std::chrono::steady_clock::now();
  auto done = [&](int rc) {
    ctx->t_take_rays = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count();
    return rc;
  };
  if (!ctx->kept_dev.empty()) {  // device-resident chunks: one pass through the pinned ring
    std::vector<D2HSeg> segs;
    for (auto& k : ctx->kept_dev) {
      segs.push_back({(const char*)k.d, (char*)(ray_xy + 2 * off), (size_t)k.npts * 16});
      off += k.npts;
    }
    HIPCHK(hipSetDevice(ctx->device));
    const int rc = d2h_pageable(ctx, segs);
    release_kept_rays(ctx);
    return done(rc);
  }
  for (auto& r : ctx->kept_rays) {
    std::copy(r.begin(), r.end(), ray_xy + 2 * off);
    off += (int64_t)r.size() / 2;
  }
  release_kept_rays(ctx);
  return done(ALIFMM_OK);
}

int alifmm_put_field(alifmm_ctx* ctx, int slot, int subgrid, const double* data) {
  if (!ctx || !ctx->have_model || slot < 0 || !data) return fail(ctx, ALIFMM_E_ARG, "put_field: bad args");
  int fz, fx;
  int rc = alifmm_field_shape(ctx, subgrid, &fz, &fx);
  if (rc) return rc;
  HIPCHK(hipSetDevice(ctx->device));
  if ((rc = af_ensure_field(ctx, slot, subgrid, fz, fx))) return rc;
  HIPCHK(hipMemcpy(ctx->fields[slot].d, data, (size_t)fz * fx * 8, hipMemcpyHostToDevice));
  return ALIFMM_OK;
}

int alifmm_time_between_points(alifmm_ctx* ctx, int n, const double* x1, const double* x2, const double* y1,
                               const double* y2, int subgrid, double* out) {
  if (!ctx || !ctx->have_model || n < 0 || subgrid < 1) return fail(ctx, ALIFMM_E_ARG, "time_between_points: bad args");
  if (n == 0) return ALIFMM_OK;
  HIPCHK(hipSetDevice(ctx->device));
  double* d = nullptr;
  HIPCHK(dalloc(&d, (size_t)5 * n));
  hipError_t e = hipSuccess;
  const double* src[4] = {x1, x2, y1, y2};
  for (int k = 0; k < 4 && e == hipSuccess; k++) e = hipMemcpy(d + (size_t)k * n, src[k], 8 * (size_t)n, hipMemcpyHostToDevice);
  af::DevModel M = dev_model(ctx);
  if (e == hipSuccess) e = af_launch_tbp(&M, n, d, d + n, d + 2 * n, d + 3 * n, ctx->dnx, subgrid, d + 4 * n, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) e = hipMemcpy(out, d + 4 * (size_t)n, 8 * (size_t)n, hipMemcpyDeviceToHost);
  dfree(d);
  if (e != hipSuccess) return fail(ctx, ALIFMM_E_HIP, "time_between_points: %s", hipGetErrorString(e));
  return ALIFMM_OK;
}

int alifmm_local_ops(alifmm_ctx* ctx, int op, int n, int pz, int px, const double* ttn, const int32_t* nsts,
                     const int32_t* iz, const int32_t* ix, const double* dnx, const double* dnz, const int32_t* nnz_arg,
                     const int32_t* nnx_arg, const double* cell_veln, const int64_t* cell_velpn, const double* cell_vm,
                     const int64_t* cell_stif, const double* tab, int ncol, double* out) {
  if (!ctx || (op != 0 && op != 1) || n < 0 || pz < 1 || px < 1 || ncol < 1)
    return fail(ctx, ALIFMM_E_ARG, "local_ops: bad args");
  if (n == 0) return ALIFMM_OK;
  HIPCHK(hipSetDevice(ctx->device));
  const size_t pn = (size_t)pz * px;
  std::vector<int> vp(n);
  for (int k = 0; k < n; k++) vp[k] = (int)cell_velpn[k];
  std::vector<double> st;
  if (cell_stif) {
    st.resize((size_t)5 * n);
    for (size_t k = 0; k < st.size(); k++) st[k] = (double)cell_stif[k];
  }
  // one device block: [ttn | cveln | cvm | dnx | dnz | tab | stif | out] doubles, [nsts | iz | ix | nnz | nnx | velpn] ints
  size_t nd = pn * n + 4 * (size_t)n + 361 * (size_t)ncol + st.size() + n;
  size_t ni = pn * n + 5 * (size_t)n;
  double* dd = nullptr;
  int* di = nullptr;
  HIPCHK(dalloc(&dd, nd));
  if (hipMalloc((void**)&di, ni * 4) != hipSuccess) {
    dfree(dd);
    return fail(ctx, ALIFMM_E_HIP, "local_ops: out of memory");
  }
  double* p = dd;
  af::LocalOpsParams P;
  memset(&P, 0, sizeof P);
  P.op = op;
  P.n = n;
  P.pz = pz;
  P.px = px;
  hipError_t e = hipSuccess;
  auto putd = [&](const double* h, size_t cnt) {
    double* q = p;
    if (e == hipSuccess && cnt) e = hipMemcpy(q, h, cnt * 8, hipMemcpyHostToDevice);
    p += cnt;
    return (const double*)q;
  };
  P.ttn = putd(ttn, pn * n);
  P.cveln = putd(cell_veln, n);
  P.cvm = putd(cell_vm, n);
  P.dnx = putd(dnx, n);
  P.dnz = putd(dnz ? dnz : dnx, n);
  P.tab = putd(tab, 361 * (size_t)ncol);
  P.cstif = cell_stif ? putd(st.data(), st.size()) : nullptr;
  P.out = p;
  int* q = di;
  auto puti = [&](const int32_t* h, size_t cnt) {
    int* r = q;
    if (e == hipSuccess && cnt) e = hipMemcpy(r, h, cnt * 4, hipMemcpyHostToDevice);
    q += cnt;
    return (const int*)r;
  };
  P.nsts = puti(nsts, pn * n);
  P.iz = puti(iz, n);
  P.ix = puti(ix, n);
  P.nnz_arg = puti(nnz_arg, n);
  P.nnx_arg = puti(nnx_arg, n);
  P.cvelpn = puti(vp.data(), n);
  P.ncol = ncol;
  if (e == hipSuccess) e = af_launch_local_ops(&P, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) e = hipMemcpy(out, P.out, 8 * (size_t)n, hipMemcpyDeviceToHost);
  dfree(dd);
  dfree(di);
  if (e != hipSuccess) return fail(ctx, ALIFMM_E_HIP, "local_ops: %s", hipGetErrorString(e));
  return ALIFMM_OK;
}

int alifmm_fouds18_band(alifmm_ctx* ctx, int n, int pz, int px, const double* ttn, const int32_t* nsts,
                        const int32_t* iz, const int32_t* ix, const double* dnx, const double* dnz,
                        const int32_t* nnz_arg, const int32_t* nnx_arg, const int32_t* mz, const int32_t* mx, int quant,
                        double* out) {
  if (!ctx || !ctx->have_model || n < 0 || pz < 1 || px < 1 || (quant != 0 && quant != 1))
    return fail(ctx, ALIFMM_E_ARG, "fouds18_band: bad args or no model");
  if (!ctx->d_mid || !ctx->d_mslo)
    return fail(ctx, ALIFMM_E_ARG, "fouds18_band: the model has no per-material table (too many materials)");
  for (int k = 0; k < n; k++)
    if (mz[k] < 0 || mz[k] >= ctx->nz0 || mx[k] < 0 || mx[k] >= ctx->nx0)
      return fail(ctx, ALIFMM_E_ARG, "fouds18_band: model cell %d (%d, %d) outside the grid", k, mz[k], mx[k]);
  if (n == 0) return ALIFMM_OK;
  HIPCHK(hipSetDevice(ctx->device));
  const size_t pn = (size_t)pz * px;
  // [ttn | dnx | dnz | out] doubles, [nsts | iz | ix | nnz | nnx | mz | mx] ints
  double* dd = nullptr;
  int* di = nullptr;
  HIPCHK(dalloc(&dd, pn * n + 3 * (size_t)n));
  if (hipMalloc((void**)&di, (pn * n + 6 * (size_t)n) * 4) != hipSuccess) {
    dfree(dd);
    return fail(ctx, ALIFMM_E_HIP, "fouds18_band: out of memory");
  }
  af::LocalOpsParams P;
  memset(&P, 0, sizeof P);
  P.op = 2;
  P.n = n;
  P.pz = pz;
  P.px = px;
  P.RM = dev_model(ctx);
  P.quant = quant;
  hipError_t e = hipSuccess;
  double* p = dd;
  auto putd = [&](const double* h, size_t cnt) {
    double* q = p;
    if (e == hipSuccess && cnt) e = hipMemcpy(q, h, cnt * 8, hipMemcpyHostToDevice);
    p += cnt;
    return (const double*)q;
  };
  int* q = di;
  auto puti = [&](const int32_t* h, size_t cnt) {
    int* r = q;
    if (e == hipSuccess && cnt) e = hipMemcpy(r, h, cnt * 4, hipMemcpyHostToDevice);
    q += cnt;
    return (const int*)r;
  };
  P.ttn = putd(ttn, pn * n);
  P.dnx = putd(dnx, n);
  P.dnz = putd(dnz ? dnz : dnx, n);
  P.out = p;
  P.nsts = puti(nsts, pn * n);
  P.iz = puti(iz, n);
  P.ix = puti(ix, n);
  P.nnz_arg = puti(nnz_arg, n);
  P.nnx_arg = puti(nnx_arg, n);
  P.mz = puti(mz, n);
  P.mx = puti(mx, n);
  if (e == hipSuccess) e = af_launch_local_ops(&P, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) e = hipMemcpy(out, P.out, 8 * (size_t)n, hipMemcpyDeviceToHost);
  dfree(dd);
  dfree(di);
  if (e != hipSuccess) return fail(ctx, ALIFMM_E_HIP, "fouds18_band: %s", hipGetErrorString(e));
  return ALIFMM_OK;
}

}  // extern "C"
