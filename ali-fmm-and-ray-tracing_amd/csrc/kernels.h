// kernels.h — parameter blocks and launchers shared by the kernels and the C-ABI host code.
#pragma once
#include "device_common.h"
#include "fmm_shared.h"

namespace af {

// per-source exchange block of the K-member band kernel (fmm_band_k.hip); zeroed by the host
// before each launch.  x1[member][step parity] = (step + 1) << 32 | payload words
// [Tmin lo, Tmin hi, live close cells, err << 24 | rim-list length], each written by its member
// with one sc1 store per step.
constexpr int kMaxK = 16;
struct KX {
  unsigned long long x1[kMaxK][2][4];
};

// one source of a band launch (fmm_exact_kernel / fmm_band_k_kernel); lists are split into K
// per-member slices (capL / K, capC / K) that spill the LDS lists of the band kernel
struct BandSrc {
  double* T;      // field (main grid, row-major): the result (fmm_band_k's copy-out writes it)
  double* Tb;     // the band kernel's working field (layout fmm_band_k.hip TbLayout), its two edge
                  // buffers after it
  int* S;         // status, row-major: fmm_exact_kernel's (mode 1), read by the band's hand-over
  int* Sb;        // the band kernel's status (layout fmm_band_k.hip SbLayout): far -1, known 0,
                  // close 1 + close-set slot
  int* Lin;       // mode 1: close cells handed over by fmm_exact_kernel (nl0 of them)
  int* L;         // close set: cells
  double* Lt;     // close set: T
  int* FS;        // free close-set slots
  int* A;         // accepted cells of the step
  int* C;         // claimed cells of the step
  int* Cp;        // their close-set slot (-1: far)
  double* V;      // claimed cells' new values
  int* Bl;        // claimed cells next to other members' columns
  int* Bp;        //   and their close-set slots
  int* D;         // edge cells accepted in the step (copied forward next step)
  double* Dv;     //   and their T
  int* Rx;        // claim items from other members' rim cells
  int* rimc;      // [K][2][capR] published close rim cells (packed cell)
  double* rimt;   //   and their T
  double* E;      // edge buffers [2][ecells] (4 columns per stripe, column-major: KGeom::eidx)
  KX* kx;
  double* Ts[2];  // stage grids (mode 1)
  int* Ss[2];
  int bbox[4];    // mode 1: rows / columns [z0, z1, x0, x1] of the main grid fmm_exact_kernel wrote
  long long steps[4];
  long long nupd;  // relax evaluations (cell-sweeps) in the main run
  long long t_begin, t_end;  // wall clock (100 MHz) when member 0 entered / left the band kernel
  int err;
  int nl0;
  // band profile (BandParams::prof): wall-clock ticks (100 MHz) of thread 0 of member 0 per phase
  // [Tmin + X1, accept + rim read, claim, evaluate, fallback, commit], list-size sums [close,
  // accepted, evaluated], max close, sub-phases [X1 wait, rim read, claim dedupe, drain before X1]
  long long ph[6];
  long long lsum[3];
  long long lmax;
  long long sub[4];
};

struct BandParams {
  DevModel M;
  int nsrc;
  int mode;      // 0: travel (subgrid 1, init from fmm_init_kernel); 1: travel_finer_grid
  int sg;        // subgrid size (mode 1)
  int nz, nx;    // main grid (fine grid in mode 1)
  double dnx, dnz;
  double cdelta, vmax, r0;
  double cdelta_far, r_far;  // band width beyond r_far nodes (0: off), ramped in over r_far .. 2 r_far
  double tstop;  // mode 1: the exact main-loop prefix stops when the heap root reaches it (fmm_exact_kernel)
  int exact_r;   // mode 1: tstop = (stage-2 half-width + exact_r) dnx / vmax (fmm_exact_lds: its window)
  int capL, capC, capS;  // list capacities, stage-grid capacity (cells)
  BandSrc* src;
  const HandoverOut* ho;  // mode 0
  const double* scx;
  const double* scz;
  double gox, goz;
  int prof;  // record BandSrc::ph / lsum (thread 0 reads the wall clock after each barrier)
  int coop;  // 1: hipLaunchCooperativeKernel (default); 0: plain launch after a residency check (under rocprofv3)
  int K;     // fmm_band_k: members per source (power of two <= kMaxK)
  int wlog;  // fmm_band_k: stripe width log2
  int capR;  // fmm_band_k: rim-list capacity per member and parity
  long ecells;  // fmm_band_k: cells per edge buffer
  int tb_pitch;   // fmm_band_k: working-field pitch (bricks per brick row, or row pitch)
  long tb_cells;  // fmm_band_k: working-field size in doubles (the edge buffers follow)
  int sb_pitch;   // fmm_band_k: status-array pitch
  long max_steps;  // fmm_band_k: a band still running after this many steps stops with error 8
  // fmm_band_k, mode 0: stream final tiles to the host while the band runs (hs null: off).  A tile
  // is W (stripe width) columns x 2^tr_log rows of one member's stripe; it is final once all its
  // cells are known (a per-member LDS counter).  Member m = src * K + member owns rslots slots of
  // W << tr_log doubles in hs (coherent pinned host memory); its i-th final tile goes to slot
  // i mod rslots (row-major, row pitch W), then entry i = (i + 1) << 32 | tz * nstripes + stripe
  // to its host queue hq + m * qcap; the slot is reused once hcons[m] (host-written: tiles taken)
  // exceeds i
  double* hs;
  unsigned long long* hq;
  const unsigned* hcons;
  int qcap;
  int rslots;
  int tr_log;  // tile rows log2 (own tiles per member <= 1024, <= 32768 cells a tile)
};

struct RayJob {
  const double* ttf;  // receiver travel-time field on the fine grid (row-major, fnz x fnx)
  double sx, sy;      // source (fine-grid x, z)
  double rx, ry;      // receiver (fine-grid x, z)
};

struct RayParams {
  DevModel M;  // coarse model (veln f64, velpn, vel_map f64, stiffness)
  int fnz, fnx;
  int sg;
  double dnx;
  int nrays;
  int max_pts;
  const RayJob* jobs;
  double* ray_x;  // [nrays][max_pts]
  double* ray_y;
  int* ray_len;
  double* times;
  int* flags;     // bit0 early exit ("Travel time to receiver increasing"), bit1 capacity, bit2 empty plane
  int glanes;     // lanes per ray (af_ray_group_lanes)
};

struct LocalOpsParams {
  int op;  // 0 update(), 1 fouds18_A(), 2 fouds18_A() as the band kernel runs it (resident model)
  long n;
  int pz, px;
  const double* ttn;  // [n][pz][px]
  const int* nsts;
  const int* iz;
  const int* ix;
  const double* dnx;
  const double* dnz;
  const int* nnz_arg;
  const int* nnx_arg;
  const double* cveln;  // material at the target cell, per case
  const int* cvelpn;
  const double* cvm;
  const double* cstif;  // [n][5] or nullptr (None)
  const double* tab;    // (361, ncol): phase table for update(), group table for fouds18_A()
  int ncol;
  double* out;
  // op 2: material of resident-model cell (mz, mx) under MatView::quant, through the per-material
  // record (band_mat<true>) and the precomputed slownesses DevModel::mslo (fouds18<true>)
  DevModel RM;
  const int* mz;
  const int* mx;
  int quant;
};

}  // namespace af

extern "C" {
hipError_t af_launch_init(const af::DevModel* M, af::InitJob* jobs, int njobs, af::HandoverOut* out, hipStream_t stream);
hipError_t af_launch_exact(const af::BandParams* P, hipStream_t stream);
hipError_t af_launch_exact_lds(const af::BandParams* P, hipStream_t stream);
int af_exact_lds_fits(int sg, int exact_r);  // fmm_exact_lds holds the stage grids of subgrid sg
hipError_t af_launch_band_k(const af::BandParams* P, hipStream_t stream);
int af_band_wgs_per_cu(void);  // band-kernel workgroups resident per CU (fmm_band_k.hip AF_WG_PER_CU)
// the band kernel's working-field layout: pitch and size (doubles) for an nz x nx main grid
int af_band_tb_pitch(int nx);
long af_band_tb_cells(int nz, int nx);
int af_band_sb_pitch(int nx);
long af_band_sb_cells(int nz, int nx);
// working fields -> the row-major result fields of every source of the launch
hipError_t af_launch_scale(double* T, long n, double sg, hipStream_t stream);
hipError_t af_launch_rays(const af::RayParams* P, hipStream_t stream);
int af_ray_waves_per_simd();
int af_ray_group_lanes(int sg, int packed);
hipError_t af_launch_pack_rays(const double* rx, const double* ry, const int* len, const long long* off, int nrays,
                               int max_pts, double* packed, hipStream_t stream);
hipError_t af_launch_local_ops(const af::LocalOpsParams* P, hipStream_t stream);
hipError_t af_launch_mat_slowness(const af::DevModel* M, double* out, hipStream_t stream);
hipError_t af_launch_tbp(const af::DevModel* M, int n, const double* x1, const double* x2, const double* y1,
                         const double* y2, double dnx, int sg, double* out, hipStream_t stream);
}
