// Does ocml's sincos(x) give the same bits as sin(x), cos(x)?  (device_common.h AF_SINCOS)
// build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off sincos_check.hip -o sincos_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
__global__ void k(const double* x, int n, unsigned long long* bad) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s1 = sin(x[i]), c1 = cos(x[i]), s2, c2;
  sincos(x[i], &s2, &c2);
  if (__double_as_longlong(s1) != __double_as_longlong(s2) || __double_as_longlong(c1) != __double_as_longlong(c2))
    atomicAdd(bad, 1ull);
}
int main() {
  const int n = 1 << 24;
  std::vector<double> h(n);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; i++) {  // effective angles in [-180, 360) degrees, as radians
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = ((double)(s >> 11) / 9007199254740992.0 * 540.0 - 180.0) * (M_PI / 180.0);
  }
  double* d; unsigned long long* b; unsigned long long hb = 0;
  hipMalloc(&d, n * 8); hipMalloc(&b, 8);
  hipMemcpy(d, h.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(b, &hb, 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(d, n, b);
  hipMemcpy(&hb, b, 8, hipMemcpyDeviceToHost);
  printf("sincos vs sin/cos: %llu of %d differ\n", hb, n);
  return hb != 0;
}
