// write_calib.hip — what TCC WRITE_SIZE reports for the band kernel's store shapes on gfx950
// (round-5 verdict: the kernel's scattered 4-B and 8-B stores were uncalibrated).  Every kernel
// writes into a 1 GiB buffer (far beyond L2 and the Infinity Cache), N = 8 M distinct 128-byte lines:
//   st4      one 4-byte store per line (status words, Sb)
//   st8      one 8-byte store per line (T, Tb)
//   st8sc1   one 8-byte sc1 store per line (edge buffers, rim lists)
//   st4x8    eight lanes store 4 bytes each into one 32-byte piece of a line (a status brick row)
//   st8x4    four lanes store 8 bytes each into one 32-byte piece of a line (a T brick row)
//   stream16 coalesced 16 bytes per lane over the whole buffer (the guide's exact case)
// Run under rocprofv3 --pmc WRITE_SIZE and divide each kernel's WRITE_SIZE (KB) by its line count:
// the bytes one scattered store is tallied at (tools/traffic.py reports the band kernel's writes
// in these units).  hipcc -O2 --offload-arch=gfx950 -o write_calib write_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ long line_of(long i, long lines) { return (i * 40503L) & (lines - 1); }

__global__ void st4(int* a, long lines) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < lines) a[line_of(i, lines) * 32] = (int)i;
}
__global__ void st8(double* a, long lines) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < lines) a[line_of(i, lines) * 16] = (double)i;
}
__global__ void st8sc1(double* a, long lines) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < lines)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a) + line_of(i, lines) * 16, (unsigned long long)i,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void st4x8(int* a, long lines) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if ((i >> 3) < lines) a[line_of(i >> 3, lines) * 32 + (i & 7)] = (int)i;
}
__global__ void st8x4(double* a, long lines) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if ((i >> 2) < lines) a[line_of(i >> 2, lines) * 16 + (i & 3)] = (double)i;
}
__global__ void stream16(double4* a, long n4) {
  for (long k = (long)blockIdx.x * blockDim.x + threadIdx.x; k < n4; k += (long)gridDim.x * blockDim.x)
    a[k] = double4{1.0, 2.0, 3.0, (double)k};
}

int main() {
  const long bytes = 1L << 30;
  const long lines = bytes / 128;
  void* a = nullptr;
  if (hipMalloc(&a, bytes) != hipSuccess) return 1;
  (void)hipMemset(a, 0, bytes);
  (void)hipDeviceSynchronize();
  const unsigned g1 = (unsigned)(lines / 256);
  hipLaunchKernelGGL(st4, dim3(g1), dim3(256), 0, 0, (int*)a, lines);
  hipLaunchKernelGGL(st8, dim3(g1), dim3(256), 0, 0, (double*)a, lines);
  hipLaunchKernelGGL(st8sc1, dim3(g1), dim3(256), 0, 0, (double*)a, lines);
  hipLaunchKernelGGL(st4x8, dim3(8 * g1), dim3(256), 0, 0, (int*)a, lines);
  hipLaunchKernelGGL(st8x4, dim3(4 * g1), dim3(256), 0, 0, (double*)a, lines);
  hipLaunchKernelGGL(stream16, dim3(1024 * 8), dim3(256), 0, 0, (double4*)a, bytes / 32);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"lines\": %ld, \"stream16_bytes\": %ld}\n", lines, bytes);
  (void)hipFree(a);
  return 0;
}
