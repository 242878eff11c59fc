// utils.hip — batched evaluation of single device functions (module-level API of the drop-in
// Anis_TTF_rays.py and device-level parity tests):
//   update() / fouds18_A() on independent caller-supplied neighbourhoods (:904-1410, :240-901)
//   time_between_points() on the resident model (:2835-2989)
#include "kernels.h"
#include "local_ops.h"
#include "band_common.h"

namespace af {

struct PatchField {  // caller patch; rows past pz read as nsts=-1 / ttn=0 (padded semantics)
  const double* T;
  const int* S;
  int nz, nx;
  AF_DEV int st(long z, long x) const { return z >= nz ? -1 : S[z * nx + x]; }
  AF_DEV double tt(long z, long x) const { return z >= nz ? 0.0 : T[z * nx + x]; }
};

__global__ void local_ops_kernel(LocalOpsParams P) {
  long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= P.n) return;
  const long pn = (long)P.pz * P.px;
  PatchField F{P.ttn + k * pn, P.nsts + k * pn, P.pz, P.px};
  if (P.op == 2) {  // the band kernel's fallback: fouds18<true> on the material record + mslo
    MatView v;
    v.s1z = v.s1x = v.s2 = 1;
    v.side1z = v.side1x = v.side2 = v.lo1z = v.lo1x = v.lo2z = v.lo2x = 0;
    v.quant = P.quant;
    const CellMat cm = band_mat<true>(P.RM, P.RM.mtab, P.RM.stab, v, P.mz[k], P.mx[k]);
    P.out[k] = fouds18<true>(F, P.RM, cm, P.iz[k], P.ix[k], P.dnx[k], P.dnz[k], P.nnx_arg[k], P.nnz_arg[k],
                             mat_slo(P.RM, v, P.mz[k], P.mx[k]));
    return;
  }
  DevModel M;
  M.mslo = nullptr;
  M.nz0 = 1;
  M.nx0 = 1;
  M.veln = P.cveln + k;
  M.velpn = P.cvelpn + k;
  M.vm = P.cvm + k;
  M.sidx = nullptr;
  M.stab = nullptr;
  M.gtab = P.tab;
  M.ptab = P.tab;
  M.ncol = P.ncol;
  CellMat cm;
  cm.veln = P.cveln[k];
  cm.vm = P.cvm[k];
  cm.velpn = P.cvelpn[k];
  cm.stif = P.cstif ? P.cstif + 5 * k : nullptr;
  double v;
  if (P.op == 0)
    v = update(F, M, cm, P.iz[k], P.ix[k], P.dnx[k], P.nnz_arg[k], P.nnx_arg[k]);
  else
    v = fouds18(F, M, cm, P.iz[k], P.ix[k], P.dnx[k], P.dnz[k], P.nnx_arg[k], P.nnz_arg[k]);
  P.out[k] = v;
}

__global__ void tbp_kernel(DevModel M, int n, const double* x1, const double* x2, const double* y1, const double* y2,
                           double dnx, int sg, double* out) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  out[k] = tbp(M, x1[k], x2[k], y1[k], y2[k], dnx, sg);
}

// fouds18_A()'s four stencil-family slownesses of every distinct material, for both MatView
// quantisations (sg = 1: as is; sg > 1: finer_grid_n's int32 orientation / float32 vel_map), with
// the CellMat band_mat() builds -> DevModel::mslo [nmat][2][4]
__global__ void mat_slowness_kernel(DevModel M, double* out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= 2 * M.nmat) return;
  const MatRec m = M.mtab[k >> 1];
  const bool quant = k & 1;
  CellMat c;
  c.velpn = m.velpn;
  c.veln = quant ? (double)(int)m.veln : m.veln;
  c.vm = quant ? (double)(float)m.vm : m.vm;
  c.stif = m.sidx >= 0 ? M.stab + 5 * m.sidx : nullptr;
  for (int q = 0; q < 4; q++) out[4 * k + q] = fouds18_slowness(M, c, q);
}

}  // namespace af

extern "C" hipError_t af_launch_local_ops(const af::LocalOpsParams* P, hipStream_t stream) {
  hipLaunchKernelGGL(af::local_ops_kernel, dim3((P->n + 63) / 64), dim3(64), 0, stream, *P);
  return hipGetLastError();
}

extern "C" hipError_t af_launch_tbp(const af::DevModel* M, int n, const double* x1, const double* x2, const double* y1,
                                    const double* y2, double dnx, int sg, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(af::tbp_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, *M, n, x1, x2, y1, y2, dnx, sg, out);
  return hipGetLastError();
}

extern "C" hipError_t af_launch_mat_slowness(const af::DevModel* M, double* out, hipStream_t stream) {
  if (M->nmat <= 0) return hipSuccess;
  hipLaunchKernelGGL(af::mat_slowness_kernel, dim3((2 * M->nmat + 63) / 64), dim3(64), 0, stream, *M, out);
  return hipGetLastError();
}

namespace af {
// final scaling of travel_finer_grid (:2832 ttn / subgrid_size)
__global__ void scale_kernel(double* T, long n, double inv) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) T[i] = T[i] / inv;
}
}  // namespace af

extern "C" hipError_t af_launch_scale(double* T, long n, double sg, hipStream_t stream) {
  hipLaunchKernelGGL(af::scale_kernel, dim3(2048), dim3(256), 0, stream, T, n, sg);
  return hipGetLastError();
}
