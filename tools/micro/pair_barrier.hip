// Microbenchmark (GPU box): cost of a two-workgroup barrier (one counter per pair, relaxed
// agent-scope atomics, sc1 polling) with one 512-thread workgroup per CU, 128 pairs.
// build: hipcc -O3 --offload-arch=gfx950 pair_barrier.hip -o pair_barrier
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ void pair_barrier(int* ctr, int& gen) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    gen += 2;
    long spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1L << 26)) break;  // never hang the box: give up after ~seconds
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(512) void k(int* ctrs, double* data, int iters, long long* cyc) {
  __shared__ double lds[18000];  // ~144 KB: one workgroup per CU
  const int b = blockIdx.x;
  const int pair = (b / 16) * 8 + (b % 8), mem = (b / 8) & 1;
  int* ctr = ctrs + pair * 32;
  int gen = 0;
  lds[threadIdx.x] = threadIdx.x;
  double acc = 0;
  long long t0 = wall_clock64();
  for (int it = 0; it < iters; it++) {
    // a little traffic: sc1 stores by one member, sc1 loads by the other
    double* d = data + (long)pair * 4096;
    if (mem == (it & 1)) __hip_atomic_store(d + threadIdx.x, (double)it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pair_barrier(ctr, gen);
    if (mem != (it & 1)) acc += __hip_atomic_load(d + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pair_barrier(ctr, gen);
    pair_barrier(ctr, gen);
  }
  long long t1 = wall_clock64();
  if (threadIdx.x == 0) cyc[b] = t1 - t0;
  if (acc < -1) lds[0] = acc;
  if (lds[threadIdx.x] < -1) data[0] = 0;
}

int main() {
  int nb = 256, iters = 10000;
  int* ctrs;
  double* data;
  long long* cyc;
  hipMalloc(&ctrs, 128 * 32 * 4);
  hipMemset(ctrs, 0, 128 * 32 * 4);
  hipMalloc(&data, 128L * 4096 * 8);
  hipMalloc(&cyc, nb * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  void* args[] = {&ctrs, &data, &iters, &cyc};
  hipError_t err = hipLaunchCooperativeKernel((void*)k, dim3(nb), dim3(512), args, 0, 0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> c(nb);
  hipMemcpy(c.data(), cyc, nb * 8, hipMemcpyDeviceToHost);
  long long mx = 0;
  for (auto v : c) mx = v > mx ? v : mx;
  printf("launch=%s ms=%.2f per_barrier_us=%.3f (wall clock max %.3f)\n", hipGetErrorString(err), ms,
         ms * 1e3 / (3.0 * iters), mx / 100.0 / (3.0 * iters));
  return 0;
}
