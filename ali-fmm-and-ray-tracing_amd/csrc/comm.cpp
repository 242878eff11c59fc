// comm.cpp — RCCL gather of resident travel-time fields onto one GPU over xGMI.
//
// The reference hands every finished field back to its parent process over a multiprocessing
// queue (parallel_TTF / parallel_TTF_finer_grid put [i, TTF] on queue2, Anis_TTF_rays.py:3610,
// :3659; parallel_TTF_rays :3733).  Here the fields stay resident on the GPU that computed them
// and, when a consumer wants them on one GPU, rank r sends its fields to the root with
// ncclSend / ncclRecv pairs inside one group (one message per field, no padding to equal shards).
// Two ways to form the communicator:
//   * one process driving G contexts (the drop-in's *_parallel methods): ncclCommInitAll;
//   * one process per GPU (bench.py --gpus N): ncclCommInitRank with a unique id that rank 0
//     creates and the ranks share by their own means (torch.distributed's gloo store in bench.py).
// librccl (≈570 MB) is dlopen'ed on first use only, so processes that never gather never load it.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <mutex>

#include "context.h"

namespace {

struct Rccl {
  bool ok = false;
  std::string why;
  decltype(&::ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&::ncclCommInitRank) CommInitRank = nullptr;
  decltype(&::ncclCommInitAll) CommInitAll = nullptr;
  decltype(&::ncclCommDestroy) CommDestroy = nullptr;
  decltype(&::ncclGroupStart) GroupStart = nullptr;
  decltype(&::ncclGroupEnd) GroupEnd = nullptr;
  decltype(&::ncclSend) Send = nullptr;
  decltype(&::ncclRecv) Recv = nullptr;
  decltype(&::ncclAllReduce) AllReduce = nullptr;
  decltype(&::ncclGetErrorString) ErrorString = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      r.why = std::string("dlopen librccl.so.1: ") + dlerror();
      return;
    }
    bool all = true;
    auto sym = [&](auto& fp, const char* name) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
      if (!fp) all = false;
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommInitAll, "ncclCommInitAll");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.AllReduce, "ncclAllReduce");
    sym(r.ErrorString, "ncclGetErrorString");
    r.ok = all;
    if (!all) r.why = "librccl.so.1 lacks an expected symbol";
  });
  return r;
}

}  // namespace

struct alifmm_comm {
  int nranks = 0;
  std::vector<alifmm_ctx*> ctx;  // local members (one per GPU driven by this process)
  std::vector<int> rank;         // their ranks
  std::vector<ncclComm_t> nc;
  int* dflag = nullptr;  // one process per GPU: device word of the ranks' agreement on a gather's arguments
  std::string err;
};

static int cfail(alifmm_comm* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

extern "C" {

int alifmm_comm_unique_id(char* id128) {
  Rccl& R = rccl();
  if (!R.ok || !id128) return ALIFMM_E_HIP;
  ncclUniqueId id;
  if (R.GetUniqueId(&id) != ncclSuccess) return ALIFMM_E_HIP;
  static_assert(sizeof(id) == NCCL_UNIQUE_ID_BYTES, "128-byte unique id");
  memcpy(id128, &id, sizeof id);
  return ALIFMM_OK;
}

int alifmm_comm_init_rank(alifmm_ctx* ctx, int nranks, int rank, const char* id128, alifmm_comm** out) {
  if (!ctx || !out || !id128 || nranks < 1 || rank < 0 || rank >= nranks) return ALIFMM_E_ARG;
  *out = nullptr;
  Rccl& R = rccl();
  if (!R.ok) return fail(ctx, ALIFMM_E_HIP, "RCCL unavailable: %s", R.why.c_str());
  ncclUniqueId id;
  memcpy(&id, id128, sizeof id);
  HIPCHK(hipSetDevice(ctx->device));
  ncclComm_t c = nullptr;
  const ncclResult_t e = R.CommInitRank(&c, nranks, id, rank);
  if (e != ncclSuccess) return fail(ctx, ALIFMM_E_HIP, "ncclCommInitRank: %s", R.ErrorString(e));
  alifmm_comm* m = new alifmm_comm();
  m->nranks = nranks;
  m->ctx = {ctx};
  m->rank = {rank};
  m->nc = {c};
  if (hipMalloc((void**)&m->dflag, sizeof(int)) != hipSuccess) {
    (void)R.CommDestroy(c);
    delete m;
    return fail(ctx, ALIFMM_E_HIP, "comm_init_rank: out of device memory");
  }
  *out = m;
  return ALIFMM_OK;
}

int alifmm_comm_init_all(alifmm_ctx* const* ctxs, int n, alifmm_comm** out) {
  if (!ctxs || !out || n < 1) return ALIFMM_E_ARG;
  *out = nullptr;
  for (int k = 0; k < n; k++)
    if (!ctxs[k]) return ALIFMM_E_ARG;
  Rccl& R = rccl();
  if (!R.ok) return fail(ctxs[0], ALIFMM_E_HIP, "RCCL unavailable: %s", R.why.c_str());
  std::vector<int> dev(n);
  for (int k = 0; k < n; k++) {
    dev[k] = ctxs[k]->device;
    for (int q = 0; q < k; q++)
      if (dev[q] == dev[k])
        return fail(ctxs[0], ALIFMM_E_ARG, "comm_init_all: contexts %d and %d share device %d (one GPU per rank)", q,
                    k, dev[k]);
  }
  std::vector<ncclComm_t> c(n, nullptr);
  const ncclResult_t e = R.CommInitAll(c.data(), n, dev.data());
  if (e != ncclSuccess) return fail(ctxs[0], ALIFMM_E_HIP, "ncclCommInitAll: %s", R.ErrorString(e));
  alifmm_comm* m = new alifmm_comm();
  m->nranks = n;
  m->ctx.assign(ctxs, ctxs + n);
  for (int k = 0; k < n; k++) m->rank.push_back(k);
  m->nc = c;
  *out = m;
  return ALIFMM_OK;
}

int alifmm_comm_destroy(alifmm_comm* comm) {
  if (!comm) return ALIFMM_OK;
  Rccl& R = rccl();
  for (size_t k = 0; k < comm->nc.size(); k++) {
    (void)hipSetDevice(comm->ctx[k]->device);
    if (comm->nc[k] && R.ok) (void)R.CommDestroy(comm->nc[k]);
  }
  if (comm->dflag) (void)hipFree(comm->dflag);
  delete comm;
  return ALIFMM_OK;
}

const char* alifmm_comm_last_error(alifmm_comm* comm) { return comm ? comm->err.c_str() : "no communicator"; }

// every check of one process's part of a gather (arguments, source slots, the root's destination
// slots, allocated here); 0 or an error code with comm->err set
static int gather_check(alifmm_comm* comm, int root, int subgrid, const int* first_slot, const int* count, int dst_slot,
                        const std::vector<long>& off, size_t* cells_out) {
  const int G = comm->nranks;
  size_t cells = 0;
  // field shape from the model of each local member (all ranks hold one model and subgrid)
  for (size_t k = 0; k < comm->ctx.size(); k++) {
    alifmm_ctx* ctx = comm->ctx[k];
    int fz = 0, fx = 0;
    if (alifmm_field_shape(ctx, subgrid, &fz, &fx)) return cfail(comm, ALIFMM_E_ARG, "gather_fields: %s", ctx->err.c_str());
    const size_t c = (size_t)fz * fx;
    if (cells && c != cells) return cfail(comm, ALIFMM_E_ARG, "gather_fields: members hold different grids");
    cells = c;
    const int r = comm->rank[k];
    for (int i = 0; i < count[r]; i++) {
      const int s = first_slot[r] + i;
      if (s >= (int)ctx->fields.size() || !ctx->fields[s].d || ctx->fields[s].bytes != c * sizeof(double))
        return cfail(comm, ALIFMM_E_ARG, "gather_fields: rank %d slot %d empty or of another shape", r, s);
    }
    if (r == root) {
      // the root's own fields: in place (dst_slot + off[root] == first_slot[root]) or into slots
      // disjoint from them (device-to-device copies)
      const long d0 = dst_slot + off[root], s0 = first_slot[root], n = count[root];
      if (n > 0 && d0 != s0 && std::max(d0, s0) < std::min(d0, s0) + n)
        return cfail(comm, ALIFMM_E_ARG, "gather_fields: the root's fields overlap their destination slots");
      for (long i = 0; i < off[G]; i++) {
        const int s = dst_slot + (int)i;
        if (i >= off[root] && i < off[root + 1] && d0 == s0) continue;  // in place
        if (s >= first_slot[root] && s < first_slot[root] + count[root] && d0 != s0)
          return cfail(comm, ALIFMM_E_ARG, "gather_fields: destination slot %d holds one of the root's fields", s);
      }
      // destination slots (allocated before the group and the clock: no allocation inside)
      (void)hipSetDevice(ctx->device);
      for (long i = 0; i < off[G]; i++) {
        if (i >= off[root] && i < off[root + 1] && d0 == s0) continue;
        const int rc = af_ensure_field(ctx, dst_slot + (int)i, subgrid, fz, fx);
        if (rc) return cfail(comm, rc, "gather_fields: %s", ctx->err.c_str());
      }
    }
  }
  *cells_out = cells;
  return ALIFMM_OK;
}

int alifmm_gather_fields(alifmm_comm* comm, int root, int subgrid, const int* first_slot, const int* count,
                         int dst_slot, double* ms) {
  // only a missing communicator or RCCL library returns at once; every other failed check still
  // joins the ranks' agreement below with a failing flag (a rank returning alone would leave its
  // peers blocked in the AllReduce)
  if (!comm) return ALIFMM_E_ARG;
  Rccl& R = rccl();
  if (!R.ok) return cfail(comm, ALIFMM_E_HIP, "RCCL unavailable: %s", R.why.c_str());
  const int G = comm->nranks;
  std::vector<long> off(G + 1, 0);  // root slot of rank r's first field: dst_slot + off[r]
  int rc = ALIFMM_OK;
  if (!first_slot || !count || root < 0 || root >= G || dst_slot < 0)
    rc = cfail(comm, ALIFMM_E_ARG, "gather_fields: bad arguments");
  for (int r = 0; r < G && !rc; r++) {
    if (count[r] < 0 || first_slot[r] < 0) rc = cfail(comm, ALIFMM_E_ARG, "gather_fields: rank %d count/slot", r);
    off[r + 1] = off[r] + std::max(count[r], 0);
  }
  size_t cells = 0;
  if (!rc) rc = gather_check(comm, root, subgrid, first_slot, count, dst_slot, off, &cells);
  // one process per GPU: the ranks agree on the checks before anyone posts a send or receive (a
  // rank that returned alone would leave its peers blocked in the group); min over the ranks' flags
  if (comm->ctx.size() < (size_t)G) {
    alifmm_ctx* ctx = comm->ctx[0];
    (void)hipSetDevice(ctx->device);
    const int mine = rc ? 0 : 1;
    int all = 0;
    if (hipMemcpyAsync(comm->dflag, &mine, sizeof(int), hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
      (void)hipMemsetAsync(comm->dflag, 0, sizeof(int), ctx->stream);  // still take part, with a failing flag
    const ncclResult_t e = R.AllReduce(comm->dflag, comm->dflag, 1, ncclInt32, ncclMin, comm->nc[0], ctx->stream);
    if (e != ncclSuccess) return cfail(comm, ALIFMM_E_HIP, "gather_fields: agreement: %s", R.ErrorString(e));
    if (hipMemcpyAsync(&all, comm->dflag, sizeof(int), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess)
      return cfail(comm, ALIFMM_E_HIP, "gather_fields: agreement: copy");
    if (rc) return rc;
    if (!all) return cfail(comm, ALIFMM_E_ARG, "gather_fields: another rank rejected the gather");
  } else if (rc) {
    return rc;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t k = 0; k < comm->ctx.size(); k++) {
    if (comm->rank[k] != root) continue;
    alifmm_ctx* ctx = comm->ctx[k];
    (void)hipSetDevice(ctx->device);
    for (int i = 0; i < count[root]; i++) {  // own fields not in place: device-to-device
      const int d = dst_slot + (int)off[root] + i, s = first_slot[root] + i;
      if (d == s) continue;
      if (hipMemcpyAsync(ctx->fields[d].d, ctx->fields[s].d, cells * sizeof(double), hipMemcpyDeviceToDevice,
                         ctx->stream) != hipSuccess)
        return cfail(comm, ALIFMM_E_HIP, "gather_fields: root copy");
    }
  }
  ncclResult_t e = R.GroupStart();
  for (size_t k = 0; k < comm->ctx.size() && e == ncclSuccess; k++) {
    alifmm_ctx* ctx = comm->ctx[k];
    const int r = comm->rank[k];
    (void)hipSetDevice(ctx->device);
    if (r != root) {
      for (int i = 0; i < count[r] && e == ncclSuccess; i++)
        e = R.Send(ctx->fields[first_slot[r] + i].d, cells, ncclDouble, root, comm->nc[k], ctx->stream);
    } else {
      for (int q = 0; q < G && e == ncclSuccess; q++) {
        if (q == root) continue;
        for (int i = 0; i < count[q] && e == ncclSuccess; i++)
          e = R.Recv(ctx->fields[dst_slot + off[q] + i].d, cells, ncclDouble, q, comm->nc[k], ctx->stream);
      }
    }
  }
  const ncclResult_t e2 = R.GroupEnd();
  if (e == ncclSuccess) e = e2;
  if (e != ncclSuccess) return cfail(comm, ALIFMM_E_HIP, "RCCL gather: %s", R.ErrorString(e));
  for (size_t k = 0; k < comm->ctx.size(); k++) {
    (void)hipSetDevice(comm->ctx[k]->device);
    if (hipStreamSynchronize(comm->ctx[k]->stream) != hipSuccess) return cfail(comm, ALIFMM_E_HIP, "gather: sync");
  }
  if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return ALIFMM_OK;
}

}  // extern "C"
