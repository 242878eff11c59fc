// fetch_calib.hip — what TCC FETCH_SIZE reports for the band kernel's access shape on gfx950.
// gather8: every lane reads ONE 8-byte value from its own 128-byte line (N distinct lines, each
//          read once: N x 128 bytes cross the L2 / fabric boundary if nothing is cached);
// stream16: coalesced 16-byte-per-lane reads of the same buffer size (the shape the guide's
//          "read = 2 x FETCH_SIZE" correction was measured on).
// Run under rocprofv3 --pmc FETCH_SIZE and compare each kernel's FETCH_SIZE (KB) with the bytes
// above: the ratio is the correction for that shape (tools/traffic.py uses it).
// hipcc -O2 --offload-arch=gfx950 -o fetch_calib fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void gather8(const double* __restrict__ a, long lines, double* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  // a scattered line order (odd multiplier mod 2^k) so neighbouring lanes do not share pages
  const long l = (i * 40503L) & (lines - 1);
  double v = i < lines ? a[l * 16] : 0.0;
  if (v == 12345.678) out[0] = v;
}

// two lanes per line: offsets 0 and 64 of the same 128-byte line (one request or two sectors?)
__global__ void gather8x2(const double* __restrict__ a, long lines, double* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long l = ((i >> 1) * 40503L) & (lines - 1);
  double v = (i >> 1) < lines ? a[l * 16 + (i & 1) * 8] : 0.0;
  if (v == 12345.678) out[0] = v;
}

__global__ void stream16(const double4* __restrict__ a, long n4, double* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  double s = 0.0;
  for (long k = i; k < n4; k += (long)gridDim.x * blockDim.x) {
    const double4 v = a[k];
    s += v.x + v.w;
  }
  if (s == 12345.678) out[0] = s;
}

int main() {
  const long bytes = 1L << 30;  // 1 GiB: far beyond L2 and the 256 MB Infinity Cache
  const long lines = bytes / 128;
  double* a = nullptr;
  double* out = nullptr;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(a, 0, bytes);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(gather8, dim3((unsigned)(lines / 256)), dim3(256), 0, 0, a, lines, out);
  hipLaunchKernelGGL(gather8x2, dim3((unsigned)(2 * lines / 256)), dim3(256), 0, 0, a, lines, out);
  hipLaunchKernelGGL(stream16, dim3(1024 * 8), dim3(256), 0, 0, (const double4*)a, bytes / 32, out);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"gather8_lines\": %ld, \"gather8_line_bytes\": %ld, \"stream16_bytes\": %ld}\n", lines, lines * 128,
         bytes);
  (void)hipFree(a);
  (void)hipFree(out);
  return 0;
}
