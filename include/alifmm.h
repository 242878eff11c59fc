/* alifmm.h — C-ABI of libalifmm.so, the MI355X (gfx950) ALI-FMM travel-time-field solver and
 * ray tracer.  Drop-in boundary for the hot path of the reference module Anis_TTF_rays.py
 * (WiPi-UoS/ALI-FMM-and-ray-tracing); each entry point names the reference interface it replaces.
 *
 * Conventions: every function returns 0 on success and a negative code on failure, with the
 * message available from alifmm_last_error(ctx).  Host buffers are caller-owned, C-contiguous,
 * row-major [iz][ix] (the reference's numpy layout).  Device memory is library-owned.  Calls are
 * synchronous (they return after their device work and any device->host copy completed).
 * One context drives one GPU; a context is not re-entrant (one host thread per context).
 */
#ifndef ALIFMM_H
#define ALIFMM_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct alifmm_ctx alifmm_ctx;

enum {
  ALIFMM_OK = 0,
  ALIFMM_E_HIP = -1,      /* HIP runtime error (device missing, out of memory, launch failure) */
  ALIFMM_E_ARG = -2,      /* invalid argument (shape, source outside the grid, no model) */
  ALIFMM_E_CAPACITY = -3, /* a device work list overflowed even after the automatic retry */
  ALIFMM_E_KERNEL = -4    /* a kernel reported an internal error (init heap overflow, ...) */
};

const char* alifmm_version(void);
int alifmm_device_count(int* n);

/* Create a context on HIP device `device` (index into the visible devices). */
int alifmm_ctx_create(int device, alifmm_ctx** out);
int alifmm_ctx_destroy(alifmm_ctx* ctx);
const char* alifmm_last_error(alifmm_ctx* ctx);

/* Upload the model (replaces the model arrays handed to travel()/travel_finer_grid()/find_ray():
 * Anis_TTF_rays.py:1464, :2121, :3105; stored by ALI_FMM.__init__ :3793-3862).
 *   veln     (nnz, nnx) float64  orientation [deg]
 *   velpn    (nnz, nnx) int64    material column; 0 selects the per-cell stiffness
 *   vel_map  (nnz, nnx) float64  velocity scale
 *   stif_den (nnz, nnx, 5) int64 c22, c23, c33, c44 [MPa], density [kg/m^3]; NULL = None
 *   group_tab, phase_tab (361, ncol) float64  velocity tables (ALI_FMM.velocity_dat / phase_vel)
 *   dnx, dnz grid spacing [m]; gox, goz origin [m]
 * ncol must be below 32768 (the init kernels pack velpn and ncol into one int): ALIFMM_E_ARG.    */
int alifmm_set_model(alifmm_ctx* ctx, int nnz, int nnx, const double* veln, const int64_t* velpn,
                     const double* vel_map, const int64_t* stif_den, const double* group_tab,
                     const double* phase_tab, int ncol, double dnx, double dnz, double gox, double goz);

/* Tuning: "members" (workgroups per source of the band kernel: 0 = as many as the device holds
 * for the batch, else 1 .. 16; results are bit-identical for every value), "stripe_log"
 * (column-stripe width log2 of the band kernel's ownership, 0 = automatic), "prof" (1: record the
 * band profile, alifmm_band_profile), "cdelta" (band width in units of dnx/vmax; unset, the
 * library chooses it per model: 0.5, narrowed down to 0.2 where the materials change from cell to
 * cell — fraction of neighbour pairs with different materials ("mat_jump", / subgrid) from 0.3 to
 * 0.6; get_option reads the subgrid-1 value),
 * "r0" (near-source band schedule radius in cells, default 40), "exact_r" (radius in cells of the
 * exact heap-ordered main-loop prefix, 0..48, default 20), "batch" (sources per launch, default
 * 256), "exact_lds" (subgrid > 1: 1 = the exact walk with its state in LDS, fmm_exact_lds.hip,
 * where the stage grids fit — subgrid <= 9; 0 = the HBM walk, fmm_exact.hip; bit-identical),
 * "coop" (band launch: 1 = cooperative, 0 = plain after a residency check), "cdelta_far" /
 * "r_far" (band width beyond Tmin = r_far * dnx / vmax, ramped in over r_far .. 2 r_far; default
 * 1.4 x the band width in force from 768 cells (0.7 at 0.5); a value set is never narrower than
 * the band width in force; cdelta_far 0 = one width everywhere), "far_sg" (the largest subgrid the
 * far band applies to, default 1), "stream_out" (subgrid-1 travels
 * with a host destination stream the fields out of the band kernel, alifmm_travel_into; default 1). */
int alifmm_set_option(alifmm_ctx* ctx, const char* name, double value);
/* Read an option, or "last_k" (workgroups per source of the last band launch), "n_cu"
 * (compute units of the device), "cdelta" / "cdelta_far" (the widths in force for the resident
 * model), "mat_jump" (the model's fraction of 4-neighbour cell pairs whose materials differ),
 * "vmax" (the model's fastest speed [m/s]: the exact prefix
 * covers T <= exact_r * dnx / vmax), "stream_tail_ms" and "stream_fallback" (last travel with a host
 * destination: ms from the band kernel's end to the last streamed tile copied; fields copied after
 * the launch instead of streamed), "exact_redo" (last travel, subgrid > 1: sources the LDS exact
 * walk handed to the HBM walk), "nmat" (distinct material records of the model; 0 when there are
 * more than the id table holds), "ray_lanes" (lanes per ray of the last find_rays launch: 9, 16, 32
 * or 64). */
int alifmm_get_option(alifmm_ctx* ctx, const char* name, double* value);

/* Shape of a travel-time field for subgrid size sg: (sg*(nnz-1)+1, sg*(nnx-1)+1). */
int alifmm_field_shape(alifmm_ctx* ctx, int subgrid, int* fnz, int* fnx);

/* First-arrival travel-time fields for nsrc sources (scx, scz in metres).
 * Replaces travel() :1463-2117 (subgrid == 1) and travel_finer_grid() :2120-2832 (subgrid > 1,
 * odd; the result is already divided by subgrid as at :2832).  The fields stay resident on the
 * device in slots first_slot .. first_slot+nsrc-1 (for alifmm_find_rays); if out != NULL they are
 * also copied to out (nsrc x fnz x fnx float64).  Field semantics: SURVEY/DESIGN parity contract. */
int alifmm_travel(alifmm_ctx* ctx, int subgrid, int nsrc, const double* scx, const double* scz,
                  int first_slot, double* out);

/* alifmm_travel() with a caller-owned destination per source: field i goes to dst[i] (pageable
 * host memory, fnz x fnx float64 each; e.g. rows of the (nsrc, fnz, fnx) stack of
 * ALI_FMM.update() :3870-3936, which need not be consecutive).  Subgrid 1: the band kernel
 * streams every tile of a field (one member's stripe, a few thousand cells) to a ring of coherent
 * pinned slots as soon as all its cells are final, and the context's copy threads move it on to
 * dst[i] while the band runs (option "stream_out", default 1; "stream_tail_ms" = the time from the
 * kernel's end to the last tile copied).  Otherwise (and for a field a tile of which did not
 * arrive) the fields are copied after the launch, as alifmm_copy_fields() kind 0.  The fields also
 * stay resident in slots first_slot .. first_slot+nsrc-1. */
int alifmm_travel_into(alifmm_ctx* ctx, int subgrid, int nsrc, const double* scx, const double* scz,
                       int first_slot, double* const* dst);

/* Copy a resident field to the host; release all resident fields. */
int alifmm_get_field(alifmm_ctx* ctx, int slot, double* out);
int alifmm_release_fields(alifmm_ctx* ctx);

/* Copy the resident fields of slots first_slot .. first_slot+n-1 (one shape) into dst, slot after
 * slot (the (nsrc, fnz, fnx) result stack of ALI_FMM.update() :3870-3936, which the reference's
 * workers return over queue2 :3610, :3659).  dst_kind 0: pageable host memory, copied through a
 * ring of pinned staging buffers (the DMA of one piece overlaps the host copy of the previous);
 * 1: host memory the DMA engine can write directly (pinned or registered); 2: device memory of
 * this context's GPU (e.g. a communication buffer); 3: pageable host memory registered with the
 * DMA engine for the duration of the copy (hipHostRegister), then written directly.
 * *gbps (nullable) = bytes / wall time. */
int alifmm_copy_fields(alifmm_ctx* ctx, int first_slot, int n, double* dst, int dst_kind, double* gbps);

/* Trace npairs rays (replaces find_ray() :3104-3465 incl. ray_time() :2992-3022).
 *   field_slot[k]        resident field of the RECEIVER of ray k (its subgrid is used)
 *   src_xy[2k], rec_xy[2k]  source / receiver (x, z) on that field's fine grid
 *   times[k]             ray travel time [s]
 *   ray_len[k]           number of points (>= 2)
 *   flags[k]             bit0: reference's early exit ("Travel time to receiver increasing"),
 *                        bit1: point capacity reached, bit2: empty candidate plane
 *   ray_xy (nullable)    packed points: ray k's x at ray_xy[2*off[k] + 2*i], z at +1,
 *                        off[k] = sum of ray_len[0..k-1]; capacity ray_xy_cap points.
 *                        ray_xy == NULL with ray_xy_cap == ALIFMM_KEEP_RAYS keeps the packed
 *                        points in the context for alifmm_take_rays() (exactly sized buffer).  */
#define ALIFMM_KEEP_RAYS (-1)
int alifmm_find_rays(alifmm_ctx* ctx, int npairs, const int32_t* field_slot, const double* src_xy,
                     const double* rec_xy, double* times, int32_t* ray_len, int32_t* flags,
                     double* ray_xy, int64_t ray_xy_cap);

/* Packed points kept by the last alifmm_find_rays(..., NULL, ALIFMM_KEEP_RAYS): *n_points = their
 * count (sum of ray_len); with ray_xy != NULL (capacity ray_xy_cap points) they are copied out in
 * the layout of alifmm_find_rays() and released.  Compact ray storage for full-matrix captures
 * (the reference's dense (n, n, 5(nnz+nnx)) arrays, :4286-4289, do not fit at 4096²). */
int alifmm_take_rays(alifmm_ctx* ctx, double* ray_xy, int64_t ray_xy_cap, int64_t* n_points);

/* Diagnostics of the last alifmm_travel(): per slot band steps [stage1, stage2, stage3|-, main]
 * and main-grid cell-sweeps (local-operator evaluations); device time of the last call's kernels. */
int alifmm_source_stats(alifmm_ctx* ctx, int slot, int64_t* steps4, int64_t* cell_sweeps);
int alifmm_last_timing(alifmm_ctx* ctx, double* init_ms, double* band_ms, double* total_ms);

/* Band-kernel profile of a slot's last alifmm_travel() when option "prof" is 1 (zeros otherwise):
 * out14[0..5] wall-clock ticks (100 MHz) spent by the workgroup in the step phases [Tmin, accept,
 * claim, evaluate, fallback, commit]; out14[6..8] sums over steps of the close / accepted /
 * evaluated list sizes; out14[9] the largest close set; out14[10..13] thread 0's ticks inside
 * phases: claim [neighbour + dedupe, nsts loads, list pushes], evaluate [neighbourhood loads]. */
int alifmm_band_profile(alifmm_ctx* ctx, int slot, int64_t* out14);
/* Wall clock (100 MHz ticks) at which the band kernel's first member of the slot's source started
 * and finished in the last alifmm_travel(): out2[0], out2[1] (dispatch and load-balance diagnostic). */
int alifmm_band_span(alifmm_ctx* ctx, int slot, int64_t* out2);
/* Source-init profile of source i of the last travel chunk (subgrid 1): wall-clock ticks
 * (100 MHz) of stage 1, 2, 3 and the exact main-loop prefix, their heap pops, the ticks the
 * relaxation role was busy in each, and their relaxations | fouds18_A() fallbacks << 32. */
int alifmm_init_profile(alifmm_ctx* ctx, int i, int64_t* out16);

/* Upload a host travel-time field (fine grid of `subgrid`) into a slot, e.g. for find_ray() on a
 * field computed elsewhere (find_ray's rec_TTF argument, :3105). */
int alifmm_put_field(alifmm_ctx* ctx, int slot, int subgrid, const double* data);

/* n straight-segment times on the resident model (time_between_points() :2835-2989; the
 * coordinates are fine-grid indices of `subgrid`).  ray_time() (:2992-3022) = ordered sum. */
int alifmm_time_between_points(alifmm_ctx* ctx, int n, const double* x1, const double* x2, const double* y1,
                               const double* y2, int subgrid, double* out);

/* Evaluate the local operators on n independent neighbourhoods (pz x px patches; rows past pz
 * read as nsts=-1/ttn=0, the reference's padded stage-1 semantics).  op 0: update() :904-1410
 * with the phase table; op 1: fouds18_A() :240-901 with the group table.  Material is given at
 * the target cell only (the operators read nothing else); cell_stif (n x 5) NULL = None. */
int alifmm_local_ops(alifmm_ctx* ctx, int op, int n, int pz, int px, const double* ttn, const int32_t* nsts,
                     const int32_t* iz, const int32_t* ix, const double* dnx, const double* dnz,
                     const int32_t* nnz_arg, const int32_t* nnx_arg, const double* cell_veln,
                     const int64_t* cell_velpn, const double* cell_vm, const int64_t* cell_stif,
                     const double* tab, int ncol, double* out);

/* fouds18_A() (:240-901) exactly as the band kernel evaluates it: the material of resident-model
 * cell (mz, mx) through the model's per-material record and its precomputed stencil slownesses
 * (quant 1: the subgrid > 1 view, orientation truncated to int32 and vel_map to float32, as
 * finer_grid_n does at :26-56).  Same patches and arguments as alifmm_local_ops op 1. */
int alifmm_fouds18_band(alifmm_ctx* ctx, int n, int pz, int px, const double* ttn, const int32_t* nsts,
                        const int32_t* iz, const int32_t* ix, const double* dnx, const double* dnz,
                        const int32_t* nnz_arg, const int32_t* nnx_arg, const int32_t* mz, const int32_t* mx,
                        int quant, double* out);

/* ---- RCCL gather of resident fields onto one GPU (replaces the reference's result return over
 * multiprocessing queue2: parallel_TTF :3610, parallel_TTF_finer_grid :3659, parallel_TTF_rays
 * :3733).  librccl is loaded on first use.  A communicator spans one GPU per rank:
 *   alifmm_comm_init_all   one process driving n contexts on n distinct GPUs (ranks = array order)
 *   alifmm_comm_init_rank  one process per GPU; every rank passes the same 128-byte id, made by one
 *                          rank with alifmm_comm_unique_id and shared by the caller's own means. */
typedef struct alifmm_comm alifmm_comm;
int alifmm_comm_unique_id(char* id128);
int alifmm_comm_init_rank(alifmm_ctx* ctx, int nranks, int rank, const char* id128, alifmm_comm** out);
int alifmm_comm_init_all(alifmm_ctx* const* ctxs, int n, alifmm_comm** out);
int alifmm_comm_destroy(alifmm_comm* comm);
const char* alifmm_comm_last_error(alifmm_comm* comm);
/* Every rank calls it with the same arrays (indexed by rank): rank r's resident slots
 * first_slot[r] .. first_slot[r]+count[r]-1 (fields of `subgrid`, one shape) arrive on the root as
 * resident slots dst_slot + count[0] + ... + count[r-1] + i, rank after rank (one ncclSend /
 * ncclRecv per field in one group; no padding).  The root's own fields stay in place when their
 * destination equals their slots, else they are copied device-to-device into free slots.
 * *ms (nullable) = wall time of the gather on this process. */
int alifmm_gather_fields(alifmm_comm* comm, int root, int subgrid, const int* first_slot, const int* count,
                         int dst_slot, double* ms);

#ifdef __cplusplus
}
#endif
#endif /* ALIFMM_H */
