/*
 * speedy_ml.h -- C ABI of the MI355X-native SPEEDY-ML hybrid hot path.
 *
 * Plain C: pointers, sizes and status codes; no torch or HIP C++ types.  Every
 * device pointer argument (d_*) is a gfx950 device address; every other pointer
 * is host memory owned by the caller.  Streams are passed as `void*` holding a
 * hipStream_t (NULL = the legacy default stream).  Functions return SML_OK (0)
 * or a negative SML_ERR_* code; sml_last_error() gives the message (per thread).
 *
 * Array layouts are the reference's Fortran layouts (column-major), so a Fortran
 * host passes its arrays unchanged:
 *   spectral field   v(mx2=62, nx=32)            -> 1984 doubles, m fastest
 *   grid field       g(ix=96, il=48)             -> 4608 doubles, x fastest, row 1 south
 *   grid4d           (4, 96, 48, 8)  = (var,x,y,z), var = T,u,v,q[g/kg]
 *   grid2d / precip  (96, 48)
 *   W_in             win(n, ninp)       (NetCDF file: win[win_y=ninp][win_x=n])
 *   W_out            wout(nout, ncs+n)  (NetCDF file: wout[wout_y=ncs+n][wout_x=nout])
 *   A                COO rows/cols (1-based), vals, k entries, duplicates additive
 * Batched calls take fields back to back (field stride 1984 or 4608 doubles).
 *
 * Reference interfaces replaced:
 *   sml_grid_batched     <- grid   (src/spe_spectral.f90:389-401)
 *   sml_spec_batched     <- spec   (src/spe_spectral.f90:403-414)
 *   sml_vdspec_batched   <- vdspec (src/spe_spectral.f90:416-452)
 *   sml_uvspec_batched   <- uvspec (src/spe_spectral.f90:351-387)
 *   sml_spectral_create  <- parmtr + inifft (src/spe_spectral.f90:45-192,
 *                           src/spe_subfft_fftpack.f90:1-11)
 *   sml_res_create / sml_res_load_region_*
 *                        <- trained_reservoir_prediction + read_trained_res +
 *                           allocate_res_new + mklsparse
 *                           (src/mod_reservoir.f90:1781-1884, :78-178;
 *                            src/mod_io.f90:2911-2956; src/mod_linalg.f90:10-25)
 *   sml_res_step         <- predict / predict_ml for every region on the rank
 *                           (src/mod_reservoir.f90:1416-1533, called per region from
 *                            src/parallelmain.f90:225-234)
 *   sml_exchange_assemble <- the root half of sendrecievegrid: outvec tiles into the
 *                           global grid + clips (src/mpires.f90:300-478,
 *                            src/res_domain.f90:769-804)
 *   sml_res_tile_inputs  <- the scatter half of sendrecievegrid: overlap input tiles,
 *                           SPEEDY local vectors, standardisation
 *                           (src/mpires.f90:558-751, src/res_domain.f90:1000-1293)
 *   sml_nc_read_region   <- read_trained_res (src/mod_io.f90:2911-2956), NetCDF-3
 *                           classic reader for the per-region weight files
 *   sml_nc_write_region  <- write_trained_res (src/mod_reservoir.f90:1701-1736,
 *                           src/mod_io.f90:1247-1496)
 *   sml_dyn_create       <- indyns (+ parmtr, inifft) (src/ini_indyns.f90:1-128)
 *   sml_dyn_impint       <- impint (src/ini_impint.f90:1-153, spe_matinv.f90)
 *   sml_dyn_step         <- step (src/dyn_step.f90:1-128: grtend, sptend, implic,
 *                           geop, hordif, timint; dyn_grtend.f90, dyn_sptend.f90,
 *                           dyn_implic.f90, dyn_geop.f90)
 *   sml_dyn_leapfrog     <- the step(2,2,...) loop of stloop (src/dyn_stloop.f90:43)
 *   sml_dyn_window       <- stepone + stloop of one agcm_main window (src/ini_stepone.f90,
 *                           src/dyn_stloop.f90:37-56; run_model, src/mpires.f90:1605)
 *   sml_dyn_from_grid    <- iogrid(30) (src/ppo_iogrid.f90:497-571)
 *   sml_dyn_to_grid      <- iogrid(31) (src/ppo_iogrid.f90:573-595)
 */
#ifndef SPEEDY_ML_H
#define SPEEDY_ML_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SML_OK 0
#define SML_ERR_ARG (-1)
#define SML_ERR_HIP (-2)
#define SML_ERR_NOMEM (-3)
#define SML_ERR_STATE (-4)
#define SML_ERR_IO (-5)
#define SML_ERR_FORMAT (-6)

#define SML_F32 1
#define SML_F64 2

/* T30L8 grid constants (mod_atparam.f90:9-14) */
#define SML_MX 31
#define SML_NX 32
#define SML_MX2 62
#define SML_IX 96
#define SML_IL 48
#define SML_KX 8
#define SML_SPEC_FIELD 1984 /* 62*32 doubles */
#define SML_GRID_FIELD 4608 /* 96*48 doubles */

const char *sml_last_error(void);
int sml_abi_version(void);

/* ----------------------------------------------------------------- spectral */
typedef struct sml_spectral sml_spectral;

/* parmtr(a) + inifft: builds the Gaussian latitudes, Legendre tables (T30) and the
 * Fourier matrices on the host, uploads them to the current device. */
int sml_spectral_create(double radius, sml_spectral **out);
int sml_spectral_destroy(sml_spectral *s);
/* host copies of the tables (any pointer may be NULL):
 * sia[24], wt[24], cpol[24*32*62] (cpol(mx2,nx,iy) column-major), nsh2[32] */
int sml_spectral_tables(const sml_spectral *s, double *sia, double *wt, double *cpol, int *nsh2);

/* grid: spectral -> grid for nfields fields; kcos = 1 (plain) or 2 (x 1/cos lat) */
int sml_grid_batched(sml_spectral *s, const double *d_spec, double *d_grid, int nfields, int kcos, void *stream);
/* spec: grid -> spectral */
int sml_spec_batched(sml_spectral *s, const double *d_grid, double *d_spec, int nfields, void *stream);
/* stage-level entry points (gridy / gridx / specx / specy), Fourier buffers are
 * varm(mx2=62, il=48) per field */
int sml_gridy_batched(sml_spectral *s, const double *d_spec, double *d_varm, int nfields, void *stream);
int sml_gridx_batched(sml_spectral *s, const double *d_varm, double *d_grid, int nfields, int kcos, void *stream);
int sml_specx_batched(sml_spectral *s, const double *d_grid, double *d_varm, int nfields, void *stream);
int sml_specy_batched(sml_spectral *s, const double *d_varm, double *d_spec, int nfields, void *stream);
/* vdspec: (u,v) grid -> (vor,div) spectral, kcos 2: u*1/cos, else u*1/cos^2 */
int sml_vdspec_batched(sml_spectral *s, const double *d_ug, const double *d_vg, double *d_vor, double *d_div,
                       int nfields, int kcos, void *stream);
/* uvspec: (vor,div) spectral -> (u cos, v cos) spectral */
int sml_uvspec_batched(sml_spectral *s, const double *d_vor, const double *d_div, double *d_ucos, double *d_vcos,
                       int nfields, void *stream);
/* host convenience (synchronous, one call = H2D + kernels + D2H): used by the
 * single-field drop-ins and the Fortran binding tests */
int sml_grid_host(sml_spectral *s, const double *spec, double *grid, int nfields, int kcos);
int sml_spec_host(sml_spectral *s, const double *grid, double *spec, int nfields);

/* ---------------------------------------------------------------- reservoirs */
typedef struct sml_reservoirs sml_reservoirs;

/* One context per rank: the regions listed in region_ids (0-based global region
 * numbers of a numregions decomposition, res_domain.f90:31-62), bottom level with
 * logp/precip/tisr inputs, sst input where sst_flags[i] != 0.
 *   n[i], k[i]      reservoir size and nnz of A for local region i
 *   chunk_speedy    132 (hybrid, predict) or 0 (ML-only, predict_ml)
 *   nout            136 (chunk_size_prediction)
 *   weight_dtype    SML_F32: W_in/A/W_out held as fp32 (exact for weights read from
 *                   the NF90_REAL files); SML_F64: held as fp64.  Arithmetic is fp64.
 *   leakage         reservoir%leakage (1.0 in the reference, mod_reservoir.f90:97) */
int sml_res_create(int numregions, int nlocal, const int *region_ids, const unsigned char *sst_flags,
                   const int *n, const int *k, int chunk_speedy, int nout, int weight_dtype, double leakage,
                   sml_reservoirs **out);
int sml_res_destroy(sml_reservoirs *c);
/* A reservoir context for a different reservoir of the same shape: ninp[i] given per
 * region (no geometry-derived inputs, no exchange/tiling tables), nout outputs each
 * unstandardized with mean/std slot out_index[o] (0-based, -1 = none), a local-model
 * block of chunk_speedy columns.  Used for the slab-ocean reservoir
 * (src/mod_slab_ocean_reservoir.f90: inputs averaged atmosphere + sst, outputs the
 * region's sst points, all unstandardized with the sst slot 36 -> out_index 35). */
int sml_res_create_generic(int numregions, int nlocal, const int *region_ids, const int *ninp, const int *n,
                           const int *k, int chunk_speedy, int nout, const signed char *out_index, int weight_dtype,
                           double leakage, sml_reservoirs **out);
/* predict_slab (src/mod_slab_ocean_reservoir.f90:1201-1249) for every local region:
 * x = tanh(A x + W_in feedback), outvec = W_out [local_model; x~] unstandardized, and
 * the raw outvec (before unstandardize) into d_local_model_next -- the reference's
 * local_model = outvec (:1235).  chunk_speedy must equal nout; the two local-model
 * buffers must not alias (swap them between steps). */
int sml_res_step_slab(sml_reservoirs *c, const double *d_feedback, const double *d_local_model,
                      double *d_local_model_next, double *d_outvec, void *stream);
/* ninp of local region i (from geometry + sst flag) */
int sml_res_ninp(const sml_reservoirs *c, int i, int *ninp);
/* packed feedback layout: offsets[nlocal+1] (in doubles) */
int sml_res_feedback_offsets(const sml_reservoirs *c, int64_t *offsets);
/* load region i from reference-layout host arrays (see header comment); mean/std[36] */
int sml_res_load_region_f32(sml_reservoirs *c, int i, const int *rows, const int *cols, const float *vals,
                            const float *win, const float *wout, const double *mean, const double *std);
int sml_res_load_region_f64(sml_reservoirs *c, int i, const int *rows, const int *cols, const double *vals,
                            const double *win, const double *wout, const double *mean, const double *std);
/* state x (current_state) of region i, host arrays of n doubles */
int sml_res_set_state(sml_reservoirs *c, int i, const double *x);
int sml_res_get_state(sml_reservoirs *c, int i, double *x);
/* One prediction step for every local region (predict, mod_reservoir.f90:1416):
 *   d_feedback    packed feedback vectors (sml_res_feedback_offsets)
 *   d_local_model [nlocal][chunk_speedy] standardized SPEEDY vectors (ignored if 0)
 *   d_outvec      [nlocal][nout] unstandardized outputs */
int sml_res_step(sml_reservoirs *c, const double *d_feedback, const double *d_local_model, double *d_outvec,
                 void *stream);
/* The same step in two halves, so the reservoir's share overlaps SPEEDY's window:
 * outvec = W_out(:,1:ncs) local_model + W_out(:,ncs+1:) x~ is split at column ncs
 * exactly as the reference's outvec_component_contribs (v_p + v_ml,
 * src/mod_reservoir.f90:1456-1459).
 *   begin:  x update from d_feedback, then v_ml into a context-owned buffer
 *           (~98 % of the step's bytes; needs no SPEEDY output)
 *   finish: v_p from d_local_model, outvec = v_p + v_ml, unstandardize
 * sml_res_step == begin + finish on one stream.  Each begin needs one finish
 * before the next begin (SML_ERR_STATE otherwise). */
int sml_res_step_begin(sml_reservoirs *c, const double *d_feedback, void *stream);
int sml_res_step_finish(sml_reservoirs *c, const double *d_local_model, double *d_outvec, void *stream);
/* discard a begun step (a begin without its finish, e.g. the pipelined loop's
 * next begin when the host restarts the prediction): waits for the device, then rolls
 * the state back to the one the begin read.  No-op when nothing is begun.
 * sml_res_set_state discards a begun step itself.  sml_res_step_begun: 1 while a
 * begin waits for its finish. */
int sml_res_step_cancel(sml_reservoirs *c);
int sml_res_step_begun(const sml_reservoirs *c, int *begun);
/* finish straight from SPEEDY's forecast grids: the local-model tiling of
 * sml_res_tile_local_model (res_domain.f90:1000-1031, standardize_state_vec_res
 * :1189-1293) fused into sml_res_step_finish, one launch; identical results.
 * d_local_model (may be NULL) also receives the tiled vectors. */
int sml_res_step_finish_grid(sml_reservoirs *c, const double *d_fc4d, const double *d_fc2d, double *d_local_model,
                             double *d_outvec, void *stream);
/* sml_res_step_finish_grid + sml_exchange_assemble of the same outvecs in one launch
 * (sendrecievegrid's assembly with the root's clips, src/mpires.f90:430-478): for a
 * context that holds every region in global order (one rank), where the exchange is
 * the identity.  d_outvec receives the outvecs as well; identical results. */
int sml_res_step_finish_assemble(sml_reservoirs *c, const double *d_fc4d, const double *d_fc2d,
                                 double *d_local_model, double *d_outvec, double *d_grid4d, double *d_grid2d,
                                 double *d_precip, void *stream);
/* cap on the waves of the v_ml readout issued by sml_res_step_begin (0 = one wave per
 * 8-row item, the default cap is 2048).  The cap leaves HBM headroom for SPEEDY when
 * both share CUs; on CUs of their own (sml_stream_create_cu_range) it is not needed. */
int sml_res_set_read_waves(sml_reservoirs *c, int waves);
/* The fallback paths, forced for every region -- the defaults take them only where a
 * region's structure does not fit the fast layout, and give the same bits: A and W_in
 * read from their CSR copies (SML_RES_PATH_CSR; before any region is loaded), the
 * state update one block per (region, part) instead of the balanced persistent grid
 * (SML_RES_PATH_PER_REGION), the v_p finish one thread per output instead of in
 * column groups (SML_RES_PATH_UNGROUPED_FINISH).  For tests and for a host bisecting a
 * difference; 0 restores the defaults. */
#define SML_RES_PATH_CSR 1
#define SML_RES_PATH_PER_REGION 2
#define SML_RES_PATH_UNGROUPED_FINISH 4
int sml_res_set_reference_paths(sml_reservoirs *c, int flags);
/* the number of CUs the context's launches get (its stream's CU mask; 0 = the whole
 * device): the balanced state update runs one block per CU over equal shares of all
 * local rows.  sml_res_update_balanced: 1 when the update takes that form (every
 * region's A / W_in in ELL form, n <= 7168, ninp <= 1024), 0 for the per-region form;
 * both give bit-identical states. */
int sml_res_set_update_cus(sml_reservoirs *c, int cus);
int sml_res_update_balanced(sml_reservoirs *c, int *balanced);
/* the compressed form of local region i's A and W_in the state update reads
 * (DESIGN.md §3.1): a_width = A's ELL main slots per row (0: the CSR copy),
 * a_overflow = 1 when rows of a_width + 1 entries keep their last entry in an
 * overflow list, win_q > 0 when W_in is block-diagonal with win_q rows per input (its
 * column i / win_q is computed, not read), win_ell = 1 when W_in is read in ELL form.
 * Layout only: every form gives bit-identical states. */
int sml_res_ell_layout(sml_reservoirs *c, int i, int *a_width, int *a_overflow, int *win_q, int *win_ell);
/* the form of sml_res_step_begin (predict's update + the v_ml half of the readout,
 * src/mod_reservoir.f90:1440-1455): 0 = the update grid, then the readout grid;
 * 1 = one launch, a block per region that updates its state and then streams its
 * W_out rows (k_res_begin, up to 3 blocks per CU); 2 = the same with the W_out loads
 * unrolled twice (1 block per CU).  Every form gives bit-identical states and sums.
 * The fused forms need the 17-row readout and <= 64 KB of LDS per region; otherwise
 * form 0 runs (sml_res_begin_fused says which). */
int sml_res_set_begin_mode(sml_reservoirs *c, int mode);
int sml_res_begin_fused(const sml_reservoirs *c, int *fused);
/* synchronize (src/mod_reservoir.f90:1352-1378), the spin-up of start_prediction
 * (:938-959): `length` updates x = (1-leak) x + leak tanh(A x + W_in u_t) for every
 * local region, no readout.  d_inputs holds `length` blocks in the packed feedback
 * layout, block t at d_inputs + t * stride doubles (stride >= total feedback). */
int sml_res_synchronize(sml_reservoirs *c, const double *d_inputs, int length, int64_t stride, void *stream);
/* start_prediction (src/mod_reservoir.f90:938-959): synchronize_print (:1381-1414) over
 * the first `length` blocks of d_inputs (layout as sml_res_synchronize; the reference
 * uses synclength/timestep - 1 blocks of its prediction data), then block `length`
 * copied into d_feedback.  The local model of the first step comes from SPEEDY's
 * forecast (sml_res_tile_local_model or the hybrid loop's start). */
int sml_res_start_prediction(sml_reservoirs *c, const double *d_inputs, int length, int64_t stride,
                             double *d_feedback, void *stream);
/* host convenience: H2D, step, D2H (synchronous) */
int sml_res_step_host(sml_reservoirs *c, const double *feedback, const double *local_model, double *outvec);
/* bytes of weights + state resident on the device (for roofline bookkeeping) */
int sml_res_footprint(const sml_reservoirs *c, int64_t *weight_bytes, int64_t *algorithmic_bytes_per_step);
/* timing hook: with capacity > 0, the next `capacity` sml_res_step calls record HIP
 * events around their update and readout kernels on the step's stream (0 = off).
 * sml_res_kernel_times waits for them and returns per-step milliseconds, then
 * rearms the recorder. */
int sml_res_enable_timing(sml_reservoirs *c, int capacity);
int sml_res_kernel_times(sml_reservoirs *c, float *update_ms, float *readout_ms, int max_steps, int *count);

/* ------------------------------------------------------------- exchange/tiling */
/* Global grids: d_grid4d[4*96*48*8], d_grid2d[96*48], d_precip[96*48].
 * assemble: scatter all numregions outvecs ([numregions][nout], region-major, as
 * produced by an all-gather of every rank's d_outvec) into the grids, then clip
 * q >= 1e-6 and precip < 1e-5 -> 0. */
int sml_exchange_assemble(sml_reservoirs *c, const double *d_outvec_all, double *d_grid4d, double *d_grid2d,
                          double *d_precip, void *stream);
/* tile: build the next step's inputs of every local region from the grids:
 *   feedback atmo/logp/precip entries from the overlap tile, standardized;
 *   feedback tisr entries copied from d_tisr (packed [nlocal][in2d], already
 *   standardized, may be NULL = keep); sst entries kept as they are;
 *   local_model from the SPEEDY forecast grids d_fc4d/d_fc2d, standardized
 *   (skipped when chunk_speedy == 0 or d_fc4d == NULL). */
int sml_res_tile_inputs(sml_reservoirs *c, const double *d_grid4d, const double *d_grid2d, const double *d_precip,
                        const double *d_fc4d, const double *d_fc2d, const double *d_tisr, double *d_feedback,
                        double *d_local_model, void *stream);
/* the two halves of sml_res_tile_inputs: feedback needs only the assembled grids
 * (ready before SPEEDY runs), local_model needs SPEEDY's forecast */
int sml_res_tile_feedback(sml_reservoirs *c, const double *d_grid4d, const double *d_grid2d, const double *d_precip,
                          const double *d_tisr, double *d_feedback, void *stream);
int sml_res_tile_local_model(sml_reservoirs *c, const double *d_fc4d, const double *d_fc2d, double *d_local_model,
                             void *stream);

/* --------------------------------------------------------- NetCDF weight files */
/* Reads worker_XXXX_level_1_<trial>.nc (NetCDF-3 classic / 64-bit offset) written
 * by the reference (write_trained_res).  Sizes come from the file's dimensions:
 * dims[0]=n (win_x), dims[1]=ninp (win_y), dims[2]=nout (wout_x),
 * dims[3]=ncs+n (wout_y), dims[4]=k (rows_x), dims[5]=36 (mean_x).
 * Call once with all array pointers NULL to get dims, then again with buffers.
 * Arrays are returned in the reference layouts (fp32 values as stored). */
int sml_nc_read_region(const char *path, int64_t *dims, float *win, float *wout, int *rows, int *cols, float *vals,
                       float *mean, float *std);
/* Writes the same layout (CDF-1, big-endian) -- for tests and tooling. */
int sml_nc_write_region(const char *path, int n, int ninp, int nout, int ncs_plus_n, int k, const float *win,
                        const float *wout, const int *rows, const int *cols, const float *vals, const float *mean,
                        const float *std);

/* ---------------------------------------------------------------- dynamics */
/* SPEEDY's spectral dynamical core on the device.  The context owns the
 * prognostic state in the reference's mod_dynvar layout (mod_dynvar.f90:15-27):
 *   vor, div, t, tr   complex(mx, nx, kx, 2) -> 2*8*1984 doubles each (level 1 first)
 *   ps                complex(mx, nx, 2)     -> 2*1984 doubles
 * and the forcing phis (mod_dynvar), tcorh, qcorh (mod_hdifcon), complex(mx, nx).
 * Physics grid tendencies, when given, are phys[4][kx][il][ix] = u, v, t, q
 * (the arrays phypar adds to, dyn_grtend.f90:225-226). */
typedef struct sml_dynamics sml_dynamics;

/* indyns (src/ini_indyns.f90:1-128) + parmtr/inifft; state and forcing zeroed */
int sml_dyn_create(double radius, sml_dynamics **out);
int sml_dyn_destroy(sml_dynamics *d);
/* impint(dt, alph) (src/ini_impint.f90:1-153): must precede sml_dyn_step and be
 * repeated whenever (dt, alph) changes, as stepone does (src/ini_stepone.f90:19-34) */
int sml_dyn_impint(sml_dynamics *d, double dt, double alph);
/* phis, tcorh, qcorh (host, any may be NULL = unchanged) */
int sml_dyn_set_forcing(sml_dynamics *d, const double *phis, const double *tcorh, const double *qcorh);
/* host copies in/out of the whole prognostic state (both time levels) */
int sml_dyn_set_state(sml_dynamics *d, const double *vor, const double *div, const double *t, const double *ps,
                      const double *tr);
int sml_dyn_get_state(sml_dynamics *d, double *vor, double *div, double *t, double *ps, double *tr);
/* phi(mx, nx, kx) = geop(j4) of the last step (src/dyn_geop.f90:1-33) */
int sml_dyn_get_phi(sml_dynamics *d, double *phi);
/* tendencies of the last step before time integration, 4*kx+1 spectral fields:
 * vordt | divdt | tdt | trdt | psdt (only meaningful after a dt <= 0 step: a step
 * with dt > 0 leaves the grid-point half of grtend's tendencies there) */
int sml_dyn_get_tendencies(sml_dynamics *d, double *tend);
/* device addresses of the state buffer ([vor|div|t|tr|ps] as above) and of a
 * scratch buffer sized for phys (4*kx*4608 doubles) */
int sml_dyn_state_device(sml_dynamics *d, double **d_state, double **d_phys);
/* step(j1, j2, dt, alph, rob, wil) (src/dyn_step.f90:1-128): grtend with the
 * physics tendencies d_phys (device, may be NULL = no physics), sptend, implic,
 * hordif, stratospheric drag, timint.  Asynchronous on `stream`. */
int sml_dyn_step(sml_dynamics *d, int j1, int j2, double dt, double alph, double rob, double wil,
                 const double *d_phys, void *stream);
/* nsteps x step(2, 2, dt, alph, rob, wil) -- the leapfrog loop of stloop
 * (src/dyn_stloop.f90:43) -- replayed from one captured hipGraph (re-captured
 * when (dt, alph, rob, wil, d_phys) change).  impint(dt, alph) must be current. */
int sml_dyn_leapfrog(sml_dynamics *d, int nsteps, double dt, double alph, double rob, double wil,
                     const double *d_phys, void *stream);
/* One SPEEDY window after iogrid(30), as run_model's agcm_main runs it
 * (src/mpires.f90:1605 -> at_gcm.f90): stepone (src/ini_stepone.f90:19-34:
 * step(1,1,delt/2), step(1,2,delt), with the lradsw the previous window left) and
 * nleap x step(2,2,2 delt) with stloop's clock restarted at istep = 1
 * (src/dyn_stloop.f90:37-56).  impint tables for delt/2, delt and 2 delt are built
 * (cached) first; the whole window is one hipGraph launch.  GPU physics as set by
 * sml_dyn_set_physics (no host tendencies).  Afterwards istep = 1 + nleap and
 * impint(2 delt, alph) is current. */
int sml_dyn_window(sml_dynamics *d, int nleap, double delt, double alph, double rob, double wil, void *stream);
/* iogrid(30) (src/ppo_iogrid.f90:497-571), the window entry: variables3d
 * grid4d(4, ix, il, kx) (T, u, v, q) and logp(ix, il), device, are rounded to
 * real(4), q < 0 set to 0, transformed (vdspec / spec + trunct) into time level 1;
 * the level is transformed back and d_minmax[8] (device, may be NULL) receives
 * min/max of u, v, t, q for the safety thresholds (see sml_dyn_is_safe). */
int sml_dyn_from_grid(sml_dynamics *d, const double *d_grid4d, const double *d_logp, double *d_minmax,
                      void *stream);
/* iogrid(31) (src/ppo_iogrid.f90:573-595), the window exit: level 1 -> grid4d, logp */
int sml_dyn_to_grid(sml_dynamics *d, double *d_grid4d, double *d_logp, void *stream);
/* is_safe_to_run_speedy from the 8 min/max values (src/ppo_iogrid.f90:563-577); a NaN
 * makes the state unsafe */
int sml_dyn_is_safe(const double *minmax);
/* run_model (src/mpires.f90:1516-1628) minus its file I/O: iogrid(30) of d_grid4d /
 * d_logp with the safety check, the window (as sml_dyn_window), iogrid(31) into
 * d_fc4d / d_fc2d, then q floored at 1e-6 (:1614-1616).  When the check fails,
 * agcm_main skips the integration (at_gcm.f90:37): the forecast is then the input
 * grid with q floored (run_model's copy, :1550-1553).  The check runs beside the
 * window; sml_dyn_last_safe reads its outcome.  The forecast buffers must not alias
 * the inputs.  The window runs as a replayed hipGraph with the exit captured in it,
 * keyed on d_grid4d / d_logp / d_fc4d / d_fc2d; up to four such graphs are kept, so a
 * caller alternating two or three buffer sets (ping-pong) replays one per set, and only
 * a fifth set evicts (re-captures) one. */
int sml_dyn_run_model(sml_dynamics *d, const double *d_grid4d, const double *d_logp, int nleap, double delt,
                      double alph, double rob, double wil, double *d_fc4d, double *d_fc2d, void *stream);
/* is_safe_to_run_speedy of the last sml_dyn_from_grid / sml_dyn_run_model, i.e. the
 * run_speedy flag the reference broadcasts (src/mpires.f90:721, :1623) and stops the
 * prediction loop on (src/parallelmain.f90:268-270).  Waits only for that check;
 * minmax (may be NULL) receives its 8 values. */
int sml_dyn_last_safe(sml_dynamics *d, int *safe, double *minmax);
/* CUs [first_cu, first_cu + num_cus) for the safety check that runs beside the
 * window (iogrid(30)'s re-grid + min/max on the context's check stream); num_cus = 0
 * lets it use any CU.  The hybrid loop puts it on CUs neither SPEEDY's nor the
 * reservoir's stream uses, so its kernels never share a CU with the window's. */
int sml_dyn_set_check_cus(sml_dynamics *d, int first_cu, int num_cus);
/* the give-up time (microseconds, default 1 s) of run_model's exit waiting in-kernel
 * for the check beside the window: an exit that gives up takes its window as unsafe
 * (the forecast is the input grid) and sml_dyn_last_safe reports that window -- and
 * only that window -- unsafe.  The hybrid loop sets it with its hop timeout. */
int sml_dyn_set_check_timeout(sml_dynamics *d, int64_t microseconds);
/* the step kernels' form: 1 (default) the fused step -- two launches per leapfrog step,
 * a*b + c contracted into FMAs, within 1e-13 of the reference's window; 0 the 8/9-launch
 * step whose Fourier transforms are FFTPACK's separate multiplies and adds, bit-exact
 * with the reference's rfftb / rfftf (the two agree to rounding, 1e-11 after 6 steps).
 * Takes effect at the next step / window. */
int sml_dyn_set_fused(sml_dynamics *d, int fused);
/* the check's stream (NULL before sml_dyn_set_check_cus or the first check): work a
 * host enqueues there runs before the next window's check */
int sml_dyn_check_stream(const sml_dynamics *d, void **stream);
/* synchronous host-buffer variants */
int sml_dyn_from_grid_host(sml_dynamics *d, const double *grid4d, const double *logp, double *minmax, int *safe);
int sml_dyn_to_grid_host(sml_dynamics *d, double *grid4d, double *logp);
/* synchronous variant taking host physics tendencies (may be NULL) */
int sml_dyn_step_host(sml_dynamics *d, int j1, int j2, double dt, double alph, double rob, double wil,
                      const double *phys);

/* ---------------------------------------------------------------- physics */
/* phypar on the GPU (src/phy_phypar.f90:1-228 with convmf, lscond, cloud, radsw,
 * radlw, suflux, vdifsc; icsea = 0, lrandf and sppt off as in the hybrid runs).
 * bc: host [15][ix*il] boundary fields in this order -- fmask1, phis0 (mod_surfcon),
 * stl_am, sst_am, soilw_am (mod_var_land/sea), alb_l, alb_s, albsfc, snowc, fsol,
 * ozone, ozupp, zenit, stratz (mod_radcon), forog (mod_sflcon).  Once set, every
 * step computes the physics of time level 1 on the GPU (dyn_grtend.f90:223-226)
 * and d_phys arguments must be NULL; bc = NULL switches it off.  Call again when the
 * fields change (the coupler / sol_oz run once a day, ini_fordate.f90). */
int sml_dyn_set_physics(sml_dynamics *d, const double *bc);
/* the slab ocean's SST in the window (run_model's sst_hybrid, src/mpires.f90:1576-1584,
 * applied by agcm_init's ini_sea, src/cpl_sea.f90:38-46): sst_am = the hybrid SST where
 * the coupler's sst_am (bc's, ice-blended as sea2atm leaves it) is < 6 K above it, +
 * sst_bias, then blended with the sea ice (sice, tice).  d_sst_grid(96, 48) device,
 * read on `stream`; NULL restores the coupler's field.  Kept in force across
 * sml_dyn_set_physics calls until replaced. */
int sml_dyn_set_hybrid_sst(sml_dynamics *d, const double *d_sst_grid, double sst_bias, void *stream);
/* sea-ice fraction / temperature sice_am, tice_am (host [ngp]; NULL = no ice) */
int sml_dyn_set_sea_ice(sml_dynamics *d, const double *sice, const double *tice);
int sml_dyn_get_sea_ice(sml_dynamics *d, double *sice, double *tice);
/* host copies of the boundary fields [15][ngp] (sml_dyn_set_physics order) and of the
 * forcing phis / tcorh / qcorh (any may be NULL) as the next window reads them */
int sml_dyn_get_physics(sml_dynamics *d, double *bc);
int sml_dyn_get_forcing(sml_dynamics *d, double *phis, double *tcorh, double *qcorh);
/* ---- the window's date-driven forcing.  run_model passes each window its calendar
 * date (src/mpires.f90:1545, :1595-1598) and agcm_init rebuilds the forcing before
 * stepone (src/ini_agcm_init.f90:57-89): newdate(0) (src/mod_date.f90:17-79),
 * ini_coupler(2) (src/cpl_main_interface.f90:1-25, cpl_land.f90:1-95, cpl_sea.f90:
 * 1-200 with icland 1, icsea 0, icice 1, isstan 0), ini_sea's hybrid SST, fordate(0)
 * (src/ini_fordate.f90:1-115); agcm_1day's fordate(1) (src/at_gcm.f90:84) repeats it
 * with the same inputs.
 * surface: host [3][ngp] = fmask_l (mod_cli_land), fmask_s (mod_cli_sea), alb0
 * (mod_surfcon) as inbcon leaves them (src/ini_inbcon.f90:38-70, 140-156). */
int sml_dyn_set_surface(sml_dynamics *d, const double *surface);
/* monthly climatologies, host [5][12][ngp] = stl12, snowd12, soilw12 (mod_cli_land),
 * sst12, sice12 (mod_cli_sea), January first (src/ini_inbcon.f90:71-230).  NULL: the
 * coupler's fields stay as sml_dyn_set_physics / sml_dyn_set_sea_ice set them. */
int sml_dyn_set_climatology(sml_dynamics *d, const double *clim);
/* the forcing of a window at (iyear, imonth, iday), on `stream` before the window:
 * with a climatology the coupler at that date (stl_am, soilw_am, snow depth, sst_am,
 * sice_am, tice_am), the hybrid SST if set (sml_dyn_set_hybrid_sst), then fordate:
 * sol_oz(tyear), snowc / alb_l / alb_s / albsfc, tcorh = spec(gamlat phis0), qcorh =
 * spec(refrh1 (qref - qsfc)) from the current stl_am / sst_am.  Skipped when neither
 * the date nor any input (the setters above, set_physics / set_sea_ice / set_forcing /
 * set_hybrid_sst) changed since the last call; _ex with force != 0 recomputes. */
int sml_dyn_fordate(sml_dynamics *d, int iyear, int imonth, int iday, void *stream);
int sml_dyn_fordate_ex(sml_dynamics *d, int iyear, int imonth, int iday, int force, void *stream);
/* fordate recomputations issued so far (skipped calls not counted) */
int sml_dyn_fordate_count(const sml_dynamics *d, int *count);
/* stloop's clock (dyn_stloop.f90:37-56): istep and mod_lflags' lradsw.  sml_dyn_step
 * uses lradsw as it stands; sml_dyn_leapfrog sets lradsw = (mod(istep, 3) == 1)
 * before each step and advances istep, as stloop does.  Initial: istep 1, lradsw 1. */
int sml_dyn_set_clock(sml_dynamics *d, int istep, int lradsw);
int sml_dyn_get_clock(const sml_dynamics *d, int *istep, int *lradsw);
/* radiation state kept between steps (mod_radcon tau2, stratc; mod_physvar tt_rsw,
 * ssrd), host [4*kx*ngp tau2 | 2*ngp stratc | kx*ngp tt_rsw | ngp ssrd], layouts
 * [band][k][ngp], [2][ngp], [k][ngp]; NULL to set = zero */
int sml_dyn_set_rad_state(sml_dynamics *d, const double *rad);
int sml_dyn_get_rad_state(sml_dynamics *d, double *rad);
/* phypar alone on grid inputs (the arrays phypar builds, phy_phypar.f90:54-66):
 * ug1, vg1, tg1, qg1, phig1 [kx][ngp] (k = 1 top), pslg1 [ngp]; tendencies
 * d_tend [4][kx][ngp] = u, v, t, q.  Uses and updates the radiation state. */
int sml_dyn_phypar(sml_dynamics *d, const double *d_ug1, const double *d_vg1, const double *d_tg1,
                   const double *d_qg1, const double *d_phig1, const double *d_pslg1, int lradsw, double *d_tend,
                   void *stream);
int sml_dyn_phypar_host(sml_dynamics *d, const double *ug1, const double *vg1, const double *tg1, const double *qg1,
                        const double *phig1, const double *pslg1, int lradsw, double *tend);
/* host forcing helpers: sol_oz(tyear) (src/phy_radiat.f90:1-121) -> fields5
 * [5][ngp] = fsol, ozone, ozupp, zenit, stratz; sflset (src/phy_suflux.f90:358-382)
 * phi0 [ngp] -> forog [ngp] */
int sml_dyn_sol_oz(const sml_dynamics *d, double tyear, double *fields5);
int sml_phys_sflset(const double *phi0, double *forog);

/* ---------------------------------------------------------------- training */
/* W_out ridge training for a batch of regions (one vertical level each).
 *   chunking_matmul  (src/mod_reservoir.f90:1643-1699): G += S S^T, B += T S^T
 *   fit_chunk_hybrid (src/mod_reservoir.f90:1233-1332) / fit_chunk_ml (:1175-1231):
 *                    regularisation + mldivide (src/mod_linalg.f90:109-151)
 * naug[i] = chunk_size_speedy + n (hybrid) or n (ML only); nout = 136.
 * Device memory: nlocal x npad^2 doubles of Gram (npad = max naug rounded up to
 * 128), so batch the regions to fit HBM (e.g. 144 regions of 6300 = 47 GB). */
typedef struct sml_train sml_train;
int sml_train_create(int nlocal, const int *naug, int nout, sml_train **out);
int sml_train_destroy(sml_train *t);
/* zero the accumulators (a new training run; sml_train_solve consumes them) */
int sml_train_reset(sml_train *t, void *stream);
/* one chunking_matmul batch of m time steps for every region:
 *   d_states : per region augmented_states(naug_i, m), column-major, back to back
 *   d_targets: per region targetdata(nout, m), column-major, back to back */
int sml_train_accumulate(sml_train *t, const double *d_states, const double *d_targets, int m, void *stream);
/* regularise (diag += beta_model for i < ncs, beta_res otherwise; squared and with
 * prior(i,i) = prior_val*beta_model^2 on b_trans when using_prior), solve
 * G W^T = B^T, write W_out(nout, naug_i) column-major per region back to back into
 * d_wout.  info (host, nlocal ints, may be NULL): potrf status per region (0 = ok,
 * filled when the stream completes).  Destroys the accumulators.  Stream-ordered on
 * `stream`; the forward substitution runs on a stream of the context (forked from and
 * joined back to `stream` by events inside the call, graph-capturable), without a CU mask. */
int sml_train_solve(sml_train *t, int ncs, double beta_res, double beta_model, int using_prior, double prior_val,
                    double *d_wout, int *info, void *stream);
int sml_train_npad(const sml_train *t, int *npad);
/* block columns per Cholesky panel (default 8): the in-panel steps are left-looking,
 * the trailing update after each panel right-looking at depth 128 x panel */
int sml_train_set_panel(sml_train *t, int panel);
/* host copies for tests: G (npad x npad, column-major, lower triangle valid) and
 * B(j, o) (npad x nout) of local region i */
int sml_train_get_gram(sml_train *t, int i, double *G, double *B);

/* measurement: sustained fp64 MFMA rate of the current device (TFLOP/s), from
 * back-to-back v_mfma_f64_16x16x4_f64 chains on every SIMD */
int sml_probe_mfma_f64(int iters, double *tflops);
/* the same probe with the median in-kernel core clock of the timed run (GHz): the
 * clock the chip holds under back-to-back fp64 MFMA (DVFS), against the nominal 2.4 */
int sml_probe_mfma_f64_clock(int iters, double *tflops, double *ghz);

/* ------------------------------------------------------------------ streams */
/* A HIP stream whose kernels run only on the logical CUs [first_cu, first_cu +
 * num_cus) of the current device (hipExtStreamCreateWithCUMask).  The hybrid loop
 * (no reference counterpart: the reference runs SPEEDY after every predict, serially,
 * parallelmain.f90:225-260) gives SPEEDY's latency-bound window its own CUs beside
 * the reservoir's HBM-bound update/readout, so the window's blocks neither wait for
 * LDS behind update blocks nor share a CU's memory pipeline with readout waves. */
int sml_stream_create_cu_range(int first_cu, int num_cus, void **stream);
int sml_stream_destroy(void *stream);

/* ------------------------------------------------------------ communicator */
/* RCCL communicator of the ranks of one node (one process per GPU, xGMI): replaces
 * the MPI world of startmpi (src/mpires.f90:21-37) for the one collective of the hot
 * path.  The 128-byte unique id comes from rank 0 (sml_comm_unique_id) over the
 * host's own channel, or through a file (sml_comm_create_file: rank 0 publishes it,
 * the others wait up to timeout_s seconds). */
typedef struct sml_comm sml_comm;
int sml_comm_unique_id(unsigned char *id128);
int sml_comm_create(int world, int rank, const unsigned char *id128, sml_comm **out);
int sml_comm_create_file(int world, int rank, const char *path, int timeout_s, sml_comm **out);
/* a rank descriptor without a transport (no RCCL communicator): rank `rank` of
 * `world` for sml_hybrid_create when the host moves the outvec slabs itself and
 * advances with sml_hybrid_advance_slabs; sml_comm_allgather and sml_hybrid_step
 * refuse it (SML_ERR_STATE) */
int sml_comm_create_local(int world, int rank, sml_comm **out);
int sml_comm_destroy(sml_comm *c);
int sml_comm_rank(const sml_comm *c, int *world, int *rank);
/* the all-gather's layout for `world` ranks of processor_decomposition
 * (src/res_domain.f90:31-62): each rank's outvecs zero-padded to the largest share
 * *maxc, received as [world][maxc][nout]; *contiguous = 1 when that is already global
 * region order (even shares); perm[numregions] (may be NULL) = the slab row of each
 * region.  Host only. */
int sml_exchange_plan(int numregions, int world, int *maxc, int *contiguous, int32_t *perm);
/* all-gather of equal slabs of `count` doubles: d_recv[world][count] (ncclAllGather) --
 * the outvec exchange that replaces sendrecievegrid's point-to-point gather/scatter
 * (src/mpires.f90:338-716) */
int sml_comm_allgather(sml_comm *c, const double *d_send, double *d_recv, int64_t count, void *stream);

/* ------------------------------------------------------------ hybrid loop */
/* The prediction loop of one rank (src/parallelmain.f90:204-270): predict for the
 * rank's regions -> outvec exchange -> assemble -> run_model (SPEEDY's window on the
 * GPU) -> re-tile.  res must hold this rank's processor_decomposition
 * (res_domain.f90:31-62) of comm's world (comm NULL = one rank); dyn must have its
 * state, forcing and physics set.  overlap != 0: the reservoir's update and v_ml
 * readout run beside SPEEDY's window on a second stream (identical results), with
 * SPEEDY on CUs [0, speedy_cus) when 0 < speedy_cus < CUs. */
typedef struct sml_hybrid sml_hybrid;
int sml_hybrid_create(sml_reservoirs *res, sml_dynamics *dyn, sml_comm *comm, int nleap, double delt, double alph,
                      double rob, double wil, int overlap, int speedy_cus, sml_hybrid **out);
int sml_hybrid_destroy(sml_hybrid *h);
/* caller-owned device buffers: packed feedback, local model [nlocal][ncs], local
 * outvecs [nlocal][nout], the assembled grids grid4d(4,96,48,8) / grid2d / precip,
 * SPEEDY's forecast grids fc4d / fc2d, tisr [nlocal][16] (standardized, may be NULL =
 * feedback tisr entries left as they are) */
int sml_hybrid_set_buffers(sml_hybrid *h, double *d_feedback, double *d_local_model, double *d_outvec,
                           double *d_grid4d, double *d_grid2d, double *d_precip, double *d_fc4d, double *d_fc2d,
                           const double *d_tisr);
/* the loop's calendar (get_current_time_delta_hour as run_model and get_tisr_by_date
 * call it, src/mpires.f90:1545, :1661): startyear, hours_base = traininglength +
 * prediction marker + synclength, step_hours = timestep.  Turns on the window's
 * date-driven forcing: advance t (1-based) runs sml_dyn_fordate at the date of hour
 * hours_base + t step_hours before its window (needs sml_dyn_set_surface).  Shares its
 * fields and February latch with sml_hybrid_set_tisr_table; resets the step count. */
int sml_hybrid_set_calendar(sml_hybrid *h, int startyear, int64_t hours_base, int step_hours);
/* date[4] = year, month, day, hour of the next advance's window */
int sml_hybrid_window_date(sml_hybrid *h, int *date);
/* fixed tisr inputs of the next steps ([nlocal][16] standardized) */
int sml_hybrid_set_tisr(sml_hybrid *h, const double *d_tisr);
/* get_tisr_by_date (src/mpires.f90:1644-1676): hourly global tisr fields
 * d_table[nhours][48][96] (nhours >= 8760, unstandardized; the reference's
 * full_tisr is the same year read per region and standardized, get_full_tisr,
 * src/mod_reservoir.f90:888-906); after step t the next feedback's tisr entries
 * come from hour sml_tisr_date_index(startyear, hours_base + (t-1) step_hours) of
 * the table, tiled and standardized per region.  NULL switches back to set_tisr. */
int sml_hybrid_set_tisr_table(sml_hybrid *h, const double *d_table, int nhours, int startyear, int64_t hours_base,
                              int step_hours);
/* the reference calendar's hour-of-year index (1-based) after hours_elapsed hours from
 * Jan 1 00 of startyear (get_current_time_delta_hour + numof_hours_into_year,
 * src/mod_calendar.f90:24-175, wrapped past 8760 as get_tisr_by_date does); *feb29
 * carries the SAVEd February of the reference's month table (0 at the start) */
int sml_tisr_date_index(int startyear, int64_t hours_elapsed, int *feb29, int *index);
/* get_current_time_delta_hour (src/mod_calendar.f90:24-92): date[4] = current year,
 * month, day, hour after hours_elapsed hours from Jan 1 00 of startyear, with the same
 * SAVEd-February latch *feb29.  Host only. */
int sml_calendar_delta_hour(int startyear, int64_t hours_elapsed, int *feb29, int *date);
/* the loop's copy of that latch (set_tisr_table resets it to 0): a host whose own
 * calendar calls already met a leap year sets 1, as the reference's process-wide
 * SAVEd table would hold (mod_reservoir.f90:355/632/638, mpires.f90:108/489) */
int sml_hybrid_set_feb29(sml_hybrid *h, int feb29);
int sml_hybrid_get_feb29(const sml_hybrid *h, int *feb29);
/* the tisr entries of every local region's feedback from one hour's global tisr
 * field d_tisr_grid(96, 48): overlap tile, (x - mean(34)) / std(34) */
int sml_res_tile_tisr_field(sml_reservoirs *c, const double *d_tisr_grid, double *d_feedback, void *stream);
/* the loop's main (reservoir + exchange) and side (SPEEDY) streams */
int sml_hybrid_streams(const sml_hybrid *h, void **main, void **side);
/* the CU split of the two streams: SPEEDY's CUs [0, speedy_cus) and the reservoir's
 * [speedy_cus, speedy_cus + res_cus) (one CU per 6 of the rank's regions, a multiple of
 * 8, 64..256 - speedy_cus; SML_RES_CUS overrides); both 0 without a split */
int sml_hybrid_cus(const sml_hybrid *h, int *speedy_cus, int *res_cus);
/* start_prediction's hand-over: inputs of the first step from an analysis grid and
 * a SPEEDY forecast of it (src/mod_reservoir.f90:938-959) */
int sml_hybrid_start(sml_hybrid *h, const double *d_grid4d, const double *d_grid2d, const double *d_precip,
                     const double *d_fc4d, const double *d_fc2d);
/* a step in two halves around a host-provided exchange: predict leaves the local
 * outvecs in d_outvec on the main stream; advance takes every region's outvecs in
 * global region order ([numregions][nout]) */
int sml_hybrid_predict(sml_hybrid *h);
int sml_hybrid_advance(sml_hybrid *h, const double *d_outvec_all);
/* advance from the all-gather's output d_recv[world][maxc][nout] (sml_exchange_plan;
 * rank q's rows zero-padded to maxc): permuted into global region order when the
 * shares are uneven, then sml_hybrid_advance.  Replaces the root's receive loop
 * and assembly of sendrecievegrid (src/mpires.f90:389-442). */
int sml_hybrid_advance_slabs(sml_hybrid *h, const double *d_recv);
/* predict + the loop's own exchange (identity on one rank, sml_comm_allgather
 * otherwise) + advance_slabs; asynchronous */
int sml_hybrid_step(sml_hybrid *h);
/* ---- slab ocean (src/parallelmain.f90:216-249; sendrecievegrid's sst half,
 * src/mpires.f90:288-478, 575-767; run_model's sst_hybrid, :1576-1584, applied by
 * ini_sea, src/cpl_sea.f90:38-46).  slab: a generic ML-only context
 * (sml_res_create_generic, chunk_speedy 0, nout = resx*resy, out_index 35, leakage 1)
 * over exactly this rank's regions with an sst input, in order, each with the 7*in2d
 * inputs of atmo_training_data_idx (src/mod_slab_ocean_reservoir.f90:1532-1563).
 * Every step the atmo feedback's lowest level, logp, sst and tisr enter a ring of
 * timestep_slab/timestep - 1 columns; when mod(t*timestep, timestep_slab) == 0 the slab
 * reservoirs predict from the ring's mean (predict_slab_ml, :1251-1296); their sst
 * travels in the exchange rows (nout + resx*resy doubles per region, so d_outvec and a
 * host exchange use sml_hybrid_exchange_width), is assembled into wholegrid_sst with
 * base_sst_grid on land (sea_mask > 0) and the 272 K floor, enters the window's sst_am
 * (sml_dyn_set_hybrid_sst) and, standardized with the slab's sst mean / std, the atmo
 * feedback's sst entries.  d_base_sst / d_sea_mask (96, 48) device, read every slab
 * step.  Call before sml_hybrid_set_buffers; train_on_sst_anomalies and
 * non_stationary_ocn_climo (both off by default, mod_reservoir.f90:42-44) are not
 * supported. */
int sml_hybrid_set_slab(sml_hybrid *h, sml_reservoirs *slab, const double *d_base_sst, const double *d_sea_mask,
                        int timestep, int timestep_slab, double sst_bias);
/* start_prediction_slab's hand-over, after sml_hybrid_start: the slab reservoirs' sst
 * d_slab_outvec[nslab][resx*resy] (unstandardized; their states synchronized by the
 * host with sml_res_start_prediction) */
int sml_hybrid_start_slab(sml_hybrid *h, const double *d_slab_outvec);
/* doubles per region in the exchange rows: nout, or nout + resx*resy with the slab */
int sml_hybrid_exchange_width(const sml_hybrid *h, int *width);
/* device views of the slab state: wholegrid_sst(96, 48), the ring
 * [timestep_slab/timestep - 1][*ring_len], the last slab feedback and slab outvecs */
int sml_hybrid_slab_buffers(const sml_hybrid *h, const double **d_sst_grid, const double **d_ring, int *ring_len,
                            const double **d_slab_feedback, const double **d_slab_outvec);
/* the two cross-stream dependencies of the overlapped loop: SML_HOP_WAIT_VALUE (a
 * sequence number written by the producer's stream, waited for by the consumer's, as
 * CP stream memory operations), SML_HOP_EVENTS (event record + wait), SML_HOP_KERNEL
 * (the same sequence number, stored by a one-lane kernel behind the producer and
 * polled by a one-lane kernel ahead of the consumer; a wait that has not seen its
 * value after ~4 s gives up and sml_hybrid_sync returns SML_ERR_STATE), or
 * SML_HOP_AUTO (the default: kernel hops when the two streams run on disjoint CUs, i.e. speedy_cus > 0,
 * else wait-value hops; events when dispatch is serialised --
 * AMD_SERIALIZE_KERNEL or rocprofv3's counter collection -- where a waiting packet or
 * kernel could stall its queue ahead of its producer; SML_HYBRID_EVENTS=1 also
 * selects events).  In the kernel mode the v_p finish
 * and run_model's entry wait for their inputs inside their own kernels.  Drains both
 * streams before switching. */
#define SML_HOP_AUTO 0
#define SML_HOP_WAIT_VALUE 1
#define SML_HOP_EVENTS 2
#define SML_HOP_KERNEL 3
int sml_hybrid_set_hop_mode(sml_hybrid *h, int mode);
/* the give-up time of the loop's in-kernel waits (kernel hops; run_model's exit waiting
 * for its safety check, at most 1 s), microseconds; default 4 s.  A wait that gives up
 * hands its consumer NaN instead of the data it did not get (the finish's local model,
 * the entry's grid; the exit takes the window as unsafe) and marks a host-visible word:
 * the next sml_hybrid_step, sml_hybrid_run_speedy (which then also yields run = 0) or
 * sml_hybrid_sync returns SML_ERR_STATE once. */
int sml_hybrid_set_hop_timeout(sml_hybrid *h, int64_t microseconds);
int sml_hybrid_hop_mode(const sml_hybrid *h, int *requested, int *effective);
/* pipelined loop (default off): each advance also issues the NEXT step's reservoir
 * begin (update + v_ml readout of the feedback it has just tiled) on the main stream,
 * so a loop restarted after a sync does not pay one begin outside the overlap; every
 * step's outvecs, grids and forecast are bitwise those of the default loop, but after
 * a step (and a sync) the reservoir states are one update ahead (the next step's).
 * The next predict only finishes that begin. */
int sml_hybrid_set_pipelined(sml_hybrid *h, int on);
/* the exchange through the communicator's transport even at world 1 (default off): a
 * one-rank loop with an RCCL communicator (sml_comm_create at world 1) then runs
 * sml_hybrid_step's world > 1 path -- outvecs to the send slab, ncclAllGather on the
 * main stream, sml_hybrid_advance_slabs from the receive slab, separate assembly --
 * instead of the identity exchange fused into the finish.  Same results, bitwise;
 * for exercising the transport on one GPU.  Refused without a transport. */
int sml_hybrid_set_force_exchange(sml_hybrid *h, int on);
/* where a step's serial chain runs -- the v_p finish with the local-model tiling, the
 * exchange and the assembly: SML_CHAIN_TWO_STREAMS on the reservoir's (main) stream,
 * between a hop from SPEEDY's stream (the forecast) and one back (the assembled grid);
 * SML_CHAIN_SPEEDY on SPEEDY's stream right behind the window, so no hop sits on the
 * critical path (the main stream keeps the re-tiling and the reservoir begin, which
 * wait for the assembled grid and signal the finish); SML_CHAIN_AUTO (default) is the
 * two-stream form (measured faster at world 1 and in an 8-rank share).
 * Bitwise the same results.  Drains both streams. */
#define SML_CHAIN_AUTO 0
#define SML_CHAIN_TWO_STREAMS 1
#define SML_CHAIN_SPEEDY 2
int sml_hybrid_set_chain(sml_hybrid *h, int mode);
int sml_hybrid_chain(const sml_hybrid *h, int *requested, int *effective);
/* the stream the local outvecs are ready on after sml_hybrid_predict: a host-driven
 * exchange runs there before sml_hybrid_advance */
int sml_hybrid_exchange_stream(const sml_hybrid *h, void **stream);
/* the number of ncclAllGather calls sml_hybrid_step has issued on this loop */
int sml_hybrid_exchanges(const sml_hybrid *h, int64_t *allgathers);
/* run_speedy of the last step (0: the reference ends the prediction,
 * parallelmain.f90:268-270); waits only for that step's safety check */
int sml_hybrid_run_speedy(sml_hybrid *h, int *run);
/* wait for the issued steps; d_local_model then holds the last window's local model */
int sml_hybrid_sync(sml_hybrid *h);
/* ------------------------------------------------------------ host plumbing */
/* zeroed device allocation / free, synchronous copies (for hosts without a GPU
 * runtime binding of their own, e.g. the Fortran host) */
int sml_device_alloc(int64_t bytes, void **d_ptr);
int sml_device_free(void *d_ptr);
int sml_copy_to_device(void *d_dst, const void *src, int64_t bytes);
int sml_copy_to_host(void *dst, const void *d_src, int64_t bytes);
/* res_domain geometry of one region (getxyresextent / getoverlapindices,
 * src/res_domain.f90:123-204), 1-based: g[12] = res_xstart, res_xend, res_ystart,
 * res_yend, resx, resy, in_xstart, in_xend, in_ystart, in_yend, inx, iny */
int sml_region_geometry(int numregions, int region, int *g);
/* processor_decomposition (src/res_domain.f90:31-62): 0-based regions of rank irank */
int sml_processor_decomposition(int numregions, int numprocs, int irank, int *regions, int *count);
/* the mean / std (36 each) local region i was loaded with (host copies) */
int sml_res_mean_std(const sml_reservoirs *c, int i, double *mean, double *std);
/* row stride (>= nout) of the outvec arrays the context writes and
 * sml_exchange_assemble reads (the hybrid loop widens it for the slab ocean's sst) */
int sml_res_set_outvec_ld(sml_reservoirs *c, int ld);
/* numregions, nlocal, chunk_speedy, nout and the local region ids (any may be NULL) */
int sml_res_info(const sml_reservoirs *c, int *numregions, int *nlocal, int *chunk_speedy, int *nout,
                 int *region_ids);

#ifdef __cplusplus
}
#endif
#endif /* SPEEDY_ML_H */
