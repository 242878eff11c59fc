// dpp_check.hip — checks the DPP wave reductions of band_common.h (wave_min_full, wave_sum_full,
// wave_or_full, wave_excl_scan, bcast) against serial results on random data, 4096 waves.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../ali-fmm-and-ray-tracing_amd/csrc dpp_check.hip -o dpp_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include "band_common.h"

__global__ void k(const double* d, const int* iv, double* omin, int* osum, int* oor, int* oscan, int* otot) {
  const int w = blockIdx.x, lane = threadIdx.x;
  const double v = d[w * 64 + lane];
  const int x = iv[w * 64 + lane];
  const double m = af::wave_min_full(v);
  const int s = af::wave_sum_full(x);
  const int o = af::wave_or_full(x);
  int tot = 0;
  const int ex = af::wave_excl_scan(x, tot);
  oscan[w * 64 + lane] = ex;
  if (lane == 5) {
    omin[w] = m;
    osum[w] = s;
    oor[w] = o;
    otot[w] = tot;
  }
}

int main() {
  const int W = 4096, N = W * 64;
  std::vector<double> d(N);
  std::vector<int> iv(N);
  srand(7);
  for (int i = 0; i < N; i++) {
    d[i] = (rand() % 7 == 0) ? INFINITY : (double)rand() / RAND_MAX;
    iv[i] = rand() % 1000;
  }
  double *dd, *dm;
  int *di, *ds, *dor, *dsc, *dt;
  hipMalloc(&dd, N * 8); hipMalloc(&di, N * 4); hipMalloc(&dm, W * 8); hipMalloc(&ds, W * 4);
  hipMalloc(&dor, W * 4); hipMalloc(&dsc, N * 4); hipMalloc(&dt, W * 4);
  hipMemcpy(dd, d.data(), N * 8, hipMemcpyHostToDevice);
  hipMemcpy(di, iv.data(), N * 4, hipMemcpyHostToDevice);
  k<<<W, 64>>>(dd, di, dm, ds, dor, dsc, dt);
  std::vector<double> m(W);
  std::vector<int> s(W), o(W), sc(N), t(W);
  hipMemcpy(m.data(), dm, W * 8, hipMemcpyDeviceToHost);
  hipMemcpy(s.data(), ds, W * 4, hipMemcpyDeviceToHost);
  hipMemcpy(o.data(), dor, W * 4, hipMemcpyDeviceToHost);
  hipMemcpy(sc.data(), dsc, N * 4, hipMemcpyDeviceToHost);
  hipMemcpy(t.data(), dt, W * 4, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int w = 0; w < W; w++) {
    double mm = INFINITY;
    int ss = 0, oo = 0, run = 0;
    for (int l = 0; l < 64; l++) {
      const int i = w * 64 + l;
      mm = fmin(mm, d[i]);
      ss += iv[i];
      oo |= iv[i];
      if (sc[i] != run) bad++;
      run += iv[i];
    }
    if (mm != m[w] || ss != s[w] || oo != o[w] || t[w] != run) bad++;
  }
  printf("{\"dpp_check\": \"%s\", \"mismatches\": %ld, \"waves\": %d}\n", bad ? "FAIL" : "ok", bad, W);
  return bad ? 1 : 0;
}
