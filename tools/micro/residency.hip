// residency.hip — do two 384-thread workgroups with ~78 KB of LDS each share a CU at once?
// Launches G workgroups (default 512 = 2 per CU) that each hold LDS_BYTES of LDS and spin ~2 ms,
// recording their CU (HW_ID / XCC_ID) and start/end wall clock; prints how many started before
// the first one finished and the largest number of workgroups seen on one CU.
// hipcc -O2 --offload-arch=gfx950 -o residency residency.hip && ./residency [G] [LDS_BYTES] [THREADS]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

constexpr int kMaxLds = 160 * 1024;

// MODE 0: few registers; 1: 168 VGPRs allocated (amdgpu_num_vgpr); 2: that plus 128 B of scratch
// per lane (a private array indexed at run time)
template <int MODE>
__device__ void probe_body(long long* rec, int lds_bytes, long long spin) {
  extern __shared__ char buf[];
  const long long t0 = wall_clock64();
  if (MODE >= 1) asm volatile("v_mov_b32 v167, 0" ::: "v167");  // the band kernel's 168 VGPRs
  if (MODE == 2) {
    volatile int priv[32];
    for (int i = 0; i < 32; i++) priv[i] = i * (int)threadIdx.x;
    buf[threadIdx.x] = (char)priv[(threadIdx.x + (int)spin) & 31];
  }
  for (int i = threadIdx.x; i < lds_bytes; i += blockDim.x) buf[i] = (char)i;
  __syncthreads();
  while (wall_clock64() - t0 < spin) __builtin_amdgcn_s_sleep(10);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    rec[4 * blockIdx.x + 0] = hw;
    rec[4 * blockIdx.x + 1] = xcc;
    rec[4 * blockIdx.x + 2] = t0;
    rec[4 * blockIdx.x + 3] = wall_clock64() + buf[threadIdx.x];
  }
}
__global__ __launch_bounds__(768) void probe0(long long* rec, int lds, long long spin) { probe_body<0>(rec, lds, spin); }
__global__ __launch_bounds__(768) __attribute__((amdgpu_num_vgpr(168))) void probe1(long long* rec, int lds, long long spin) {
  probe_body<1>(rec, lds, spin);
}
__global__ __launch_bounds__(768) __attribute__((amdgpu_num_vgpr(168))) void probe2(long long* rec, int lds, long long spin) {
  probe_body<2>(rec, lds, spin);
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 512;
  const int lds = argc > 2 ? atoi(argv[2]) : 78160;
  const int thr = argc > 3 ? atoi(argv[3]) : 384;
  const int mode = argc > 4 ? atoi(argv[4]) : 0;
  const void* fn = mode == 0 ? (const void*)probe0 : mode == 1 ? (const void*)probe1 : (const void*)probe2;
  if (lds > kMaxLds) return 2;
  long long* d = nullptr;
  if (hipMalloc(&d, sizeof(long long) * 4 * G) != hipSuccess) return 1;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return 3;
  int per_cu = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, thr, lds);
  long long spin = 200000LL;  // 2 ms at 100 MHz
  void* args[] = {&d, (void*)&lds, &spin};
  if (hipLaunchKernel(fn, dim3(G), dim3(thr), args, lds, 0) != hipSuccess) return 5;
  if (hipDeviceSynchronize() != hipSuccess) return 4;
  std::vector<long long> h(4 * G);
  (void)hipMemcpy(h.data(), d, sizeof(long long) * 4 * G, hipMemcpyDeviceToHost);
  long long first_end = h[3], last_start = h[2], t_min = h[2], t_max = h[3];
  std::map<long long, int> per;
  for (int b = 0; b < G; b++) {
    first_end = std::min(first_end, h[4 * b + 3]);
    last_start = std::max(last_start, h[4 * b + 2]);
    t_min = std::min(t_min, h[4 * b + 2]);
    t_max = std::max(t_max, h[4 * b + 3]);
    const long long hw = h[4 * b], cu = ((hw >> 8) & 15) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 3) << 5);
    per[(h[4 * b + 1] & 15) << 8 | cu]++;
  }
  int started_before_first_end = 0, maxper = 0;
  for (int b = 0; b < G; b++) started_before_first_end += h[4 * b + 2] < first_end;
  for (auto& kv : per) maxper = std::max(maxper, kv.second);
  printf("{\"mode\": %d, \"grid\": %d, \"threads\": %d, \"lds\": %d, \"occupancy_per_cu\": %d, \"distinct_cus\": %zu, "
         "\"max_wgs_on_one_cu\": %d, \"started_before_first_end\": %d, \"span_ms\": %.3f}\n",
         mode, G, thr, lds, per_cu, per.size(), maxper, started_before_first_end, (t_max - t_min) / 1e5);
  (void)hipFree(d);
  return 0;
}
