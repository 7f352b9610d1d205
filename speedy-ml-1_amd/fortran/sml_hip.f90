!> sml_hip -- ISO_C_BINDING interface of libspeedyml (include/speedy_ml.h) for the
!> Fortran host of SPEEDY-ML.
!>
!> This is the binding a reference maintainer adds: the reference calls predict()
!> per region (src/parallelmain.f90:225-234 -> src/mod_reservoir.f90:1416) and the
!> external spectral routines grid/spec/vdspec/uvspec one field at a time
!> (src/spe_spectral.f90:351-452).  The interfaces below hand the same
!> column-major Fortran arrays to the batched GPU entry points.  Helper routines
!> mirror the reference's names:
!>   sml_read_trained_res  <- read_trained_res (src/mod_io.f90:2911-2956)
!>   sml_predict_all       <- predict for every region of the rank
!>   sml_check             <- nc_check-style error stop (src/mod_io.f90:1732-1744)
module sml_hip
  use iso_c_binding
  implicit none

  integer(c_int), parameter :: SML_OK = 0, SML_F32 = 1, SML_F64 = 2
  integer, parameter :: SML_SPEC_FIELD = 1984, SML_GRID_FIELD = 4608

  interface
    function sml_last_error() bind(C, name='sml_last_error') result(p)
      import :: c_ptr
      type(c_ptr) :: p
    end function
    function sml_abi_version() bind(C, name='sml_abi_version') result(v)
      import :: c_int
      integer(c_int) :: v
    end function

    ! ------------------------------------------------------------ spectral
    function sml_spectral_create(radius, ctx) bind(C, name='sml_spectral_create') result(rc)
      import :: c_double, c_ptr, c_int
      real(c_double), value :: radius
      type(c_ptr) :: ctx
      integer(c_int) :: rc
    end function
    function sml_spectral_destroy(ctx) bind(C, name='sml_spectral_destroy') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int) :: rc
    end function
    !> grid for nf fields: spec(62,32,nf) -> grid(96,48,nf) (host arrays, synchronous)
    function sml_grid_host(ctx, spec, grid, nf, kcos) bind(C, name='sml_grid_host') result(rc)
      import :: c_ptr, c_double, c_int
      type(c_ptr), value :: ctx
      real(c_double), intent(in) :: spec(*)
      real(c_double), intent(out) :: grid(*)
      integer(c_int), value :: nf, kcos
      integer(c_int) :: rc
    end function
    function sml_spec_host(ctx, grid, spec, nf) bind(C, name='sml_spec_host') result(rc)
      import :: c_ptr, c_double, c_int
      type(c_ptr), value :: ctx
      real(c_double), intent(in) :: grid(*)
      real(c_double), intent(out) :: spec(*)
      integer(c_int), value :: nf
      integer(c_int) :: rc
    end function
    !> device-pointer batched forms (arrays already resident on the GPU)
    function sml_grid_batched(ctx, d_spec, d_grid, nf, kcos, stream) bind(C, name='sml_grid_batched') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx, d_spec, d_grid, stream
      integer(c_int), value :: nf, kcos
      integer(c_int) :: rc
    end function
    function sml_spec_batched(ctx, d_grid, d_spec, nf, stream) bind(C, name='sml_spec_batched') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx, d_grid, d_spec, stream
      integer(c_int), value :: nf
      integer(c_int) :: rc
    end function

    ! ------------------------------------------------------------ reservoirs
    !> a generic context (the slab-ocean reservoirs): ninp per region, outputs
    !> unstandardized with mean / std slot out_index(o) (0-based, -1 = none)
    function sml_res_create_generic(numregions, nlocal, region_ids, ninp, n, k, chunk_speedy, nout, out_index, &
                                    weight_dtype, leakage, ctx) bind(C, name='sml_res_create_generic') result(rc)
      import :: c_int, c_signed_char, c_double, c_ptr
      integer(c_int), value :: numregions, nlocal, chunk_speedy, nout, weight_dtype
      integer(c_int), intent(in) :: region_ids(*), ninp(*), n(*), k(*)
      integer(c_signed_char), intent(in) :: out_index(*)
      real(c_double), value :: leakage
      type(c_ptr) :: ctx
      integer(c_int) :: rc
    end function
    function sml_res_create(numregions, nlocal, region_ids, sst_flags, n, k, chunk_speedy, nout, &
                            weight_dtype, leakage, ctx) bind(C, name='sml_res_create') result(rc)
      import :: c_int, c_signed_char, c_double, c_ptr
      integer(c_int), value :: numregions, nlocal, chunk_speedy, nout, weight_dtype
      integer(c_int), intent(in) :: region_ids(*), n(*), k(*)
      integer(c_signed_char), intent(in) :: sst_flags(*)
      real(c_double), value :: leakage
      type(c_ptr) :: ctx
      integer(c_int) :: rc
    end function
    function sml_res_destroy(ctx) bind(C, name='sml_res_destroy') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int) :: rc
    end function
    function sml_res_ninp(ctx, i, ninp) bind(C, name='sml_res_ninp') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int), value :: i
      integer(c_int), intent(out) :: ninp
      integer(c_int) :: rc
    end function
    function sml_res_feedback_offsets(ctx, offsets) bind(C, name='sml_res_feedback_offsets') result(rc)
      import :: c_ptr, c_int, c_int64_t
      type(c_ptr), value :: ctx
      integer(c_int64_t), intent(out) :: offsets(*)
      integer(c_int) :: rc
    end function
    !> i is 0-based; arrays in the reference layouts: win(n,ninp), wout(nout,ncs+n)
    function sml_res_load_region_f32(ctx, i, rows, cols, vals, win, wout, mean, std) &
        bind(C, name='sml_res_load_region_f32') result(rc)
      import :: c_ptr, c_int, c_float, c_double
      type(c_ptr), value :: ctx
      integer(c_int), value :: i
      integer(c_int), intent(in) :: rows(*), cols(*)
      real(c_float), intent(in) :: vals(*), win(*), wout(*)
      real(c_double), intent(in) :: mean(*), std(*)
      integer(c_int) :: rc
    end function
    function sml_res_load_region_f64(ctx, i, rows, cols, vals, win, wout, mean, std) &
        bind(C, name='sml_res_load_region_f64') result(rc)
      import :: c_ptr, c_int, c_double
      type(c_ptr), value :: ctx
      integer(c_int), value :: i
      integer(c_int), intent(in) :: rows(*), cols(*)
      real(c_double), intent(in) :: vals(*), win(*), wout(*)
      real(c_double), intent(in) :: mean(*), std(*)
      integer(c_int) :: rc
    end function
    function sml_res_set_state(ctx, i, x) bind(C, name='sml_res_set_state') result(rc)
      import :: c_ptr, c_int, c_double
      type(c_ptr), value :: ctx
      integer(c_int), value :: i
      real(c_double), intent(in) :: x(*)
      integer(c_int) :: rc
    end function
    function sml_res_get_state(ctx, i, x) bind(C, name='sml_res_get_state') result(rc)
      import :: c_ptr, c_int, c_double
      type(c_ptr), value :: ctx
      integer(c_int), value :: i
      real(c_double), intent(out) :: x(*)
      integer(c_int) :: rc
    end function
    !> predict for every local region, host buffers (PCIe-inclusive convenience)
    function sml_res_step_host(ctx, feedback, local_model, outvec) bind(C, name='sml_res_step_host') result(rc)
      import :: c_ptr, c_int, c_double
      type(c_ptr), value :: ctx
      real(c_double), intent(in) :: feedback(*), local_model(*)
      real(c_double), intent(out) :: outvec(*)
      integer(c_int) :: rc
    end function
    !> device-resident form
    function sml_res_step(ctx, d_feedback, d_local_model, d_outvec, stream) bind(C, name='sml_res_step') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx, d_feedback, d_local_model, d_outvec, stream
      integer(c_int) :: rc
    end function

    ! predict split at column chunk_size_speedy (v_ml + v_p, mod_reservoir.f90:1456-1459)
    function sml_res_step_begin(ctx, d_feedback, stream) bind(C, name='sml_res_step_begin') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx, d_feedback, stream
      integer(c_int) :: rc
    end function

    ! finish from SPEEDY's forecast grids: tile_local_model fused into the v_p finish
    function sml_res_step_finish_grid(ctx, d_fc4d, d_fc2d, d_local_model, d_outvec, stream) &
        bind(C, name='sml_res_step_finish_grid') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx, d_fc4d, d_fc2d, d_local_model, d_outvec, stream
      integer(c_int) :: rc
    end function

    ! discard a begun step (state rolled back); 1 in begun while a begin waits for its finish
    function sml_res_step_cancel(ctx) bind(C, name='sml_res_step_cancel') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int) :: rc
    end function
    function sml_res_step_begun(ctx, begun) bind(C, name='sml_res_step_begun') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int), intent(out) :: begun
      integer(c_int) :: rc
    end function

    ! the CUs the context's launches get (one balanced-update block per CU); 0 = all
    function sml_res_set_update_cus(ctx, cus) bind(C, name='sml_res_set_update_cus') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int), value :: cus
      integer(c_int) :: rc
    end function
    function sml_res_update_balanced(ctx, balanced) bind(C, name='sml_res_update_balanced') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int), intent(out) :: balanced
      integer(c_int) :: rc
    end function

    function sml_res_set_read_waves(ctx, waves) bind(C, name='sml_res_set_read_waves') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int), value :: waves
      integer(c_int) :: rc
    end function

    ! sml_res_step_begin's form: 0 update + readout grids, 1 / 2 one fused launch (bitwise the same)
    function sml_res_set_begin_mode(ctx, mode) bind(C, name='sml_res_set_begin_mode') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int), value :: mode
      integer(c_int) :: rc
    end function

    function sml_res_begin_fused(ctx, fused) bind(C, name='sml_res_begin_fused') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int) :: fused
      integer(c_int) :: rc
    end function

    ! a stream on the logical CUs [first_cu, first_cu + num_cus) (hipExtStreamCreateWithCUMask)
    function sml_stream_create_cu_range(first_cu, num_cus, stream) bind(C, name='sml_stream_create_cu_range') result(rc)
      import :: c_ptr, c_int
      integer(c_int), value :: first_cu, num_cus
      type(c_ptr) :: stream
      integer(c_int) :: rc
    end function

    function sml_stream_destroy(stream) bind(C, name='sml_stream_destroy') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: stream
      integer(c_int) :: rc
    end function

    function sml_res_step_finish(ctx, d_local_model, d_outvec, stream) bind(C, name='sml_res_step_finish') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx, d_local_model, d_outvec, stream
      integer(c_int) :: rc
    end function

    ! ------------------------------------------------------------ NetCDF weight files
    function sml_nc_read_region(path, dims, win, wout, rows, cols, vals, mean, std) &
        bind(C, name='sml_nc_read_region') result(rc)
      import :: c_char, c_int64_t, c_ptr, c_int
      character(kind=c_char), intent(in) :: path(*)
      integer(c_int64_t), intent(out) :: dims(6)
      type(c_ptr), value :: win, wout, rows, cols, vals, mean, std
      integer(c_int) :: rc
    end function

    ! ------------------------------------------------------------ SPEEDY dynamics
    !> indyns (+ parmtr/inifft); the state mirrors mod_dynvar (vor, div, t, ps, tr)
    function sml_dyn_create(radius, ctx) bind(C, name='sml_dyn_create') result(rc)
      import :: c_double, c_ptr, c_int
      real(c_double), value :: radius
      type(c_ptr), intent(out) :: ctx
      integer(c_int) :: rc
    end function
    function sml_dyn_destroy(ctx) bind(C, name='sml_dyn_destroy') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int) :: rc
    end function
    !> impint(dt, alph) (ini_impint.f90)
    function sml_dyn_impint(ctx, dt, alph) bind(C, name='sml_dyn_impint') result(rc)
      import :: c_ptr, c_double, c_int
      type(c_ptr), value :: ctx
      real(c_double), value :: dt, alph
      integer(c_int) :: rc
    end function
    !> phis (mod_dynvar), tcorh / qcorh (mod_hdifcon): complex(mx, nx)
    function sml_dyn_set_forcing(ctx, phis, tcorh, qcorh) bind(C, name='sml_dyn_set_forcing') result(rc)
      import :: c_ptr, c_double_complex, c_int
      type(c_ptr), value :: ctx
      complex(c_double_complex), intent(in) :: phis(*), tcorh(*), qcorh(*)
      integer(c_int) :: rc
    end function
    !> whole mod_dynvar state in / out: vor/div/t(mx,nx,kx,2), ps(mx,nx,2), tr(mx,nx,kx,2,1)
    function sml_dyn_set_state(ctx, vor, div, t, ps, tr) bind(C, name='sml_dyn_set_state') result(rc)
      import :: c_ptr, c_double_complex, c_int
      type(c_ptr), value :: ctx
      complex(c_double_complex), intent(in) :: vor(*), div(*), t(*), ps(*), tr(*)
      integer(c_int) :: rc
    end function
    function sml_dyn_get_state(ctx, vor, div, t, ps, tr) bind(C, name='sml_dyn_get_state') result(rc)
      import :: c_ptr, c_double_complex, c_int
      type(c_ptr), value :: ctx
      complex(c_double_complex), intent(out) :: vor(*), div(*), t(*), ps(*), tr(*)
      integer(c_int) :: rc
    end function
    !> step(j1, j2, dt, alph, rob, wil) with host physics tendencies
    !> phys(ix*il, kx, 4) = (utend, vtend, ttend, qtend) of phypar
    ! one agcm_main window: stepone + nleap leapfrog steps as one hipGraph launch
    function sml_dyn_window(ctx, nleap, delt, alph, rob, wil, stream) bind(C, name='sml_dyn_window') result(rc)
      import :: c_ptr, c_int, c_double
      type(c_ptr), value :: ctx, stream
      integer(c_int), value :: nleap
      real(c_double), value :: delt, alph, rob, wil
      integer(c_int) :: rc
    end function

    function sml_dyn_step_host(ctx, j1, j2, dt, alph, rob, wil, phys) bind(C, name='sml_dyn_step_host') result(rc)
      import :: c_ptr, c_int, c_double
      type(c_ptr), value :: ctx
      integer(c_int), value :: j1, j2
      real(c_double), value :: dt, alph, rob, wil
      real(c_double), intent(in) :: phys(*)
      integer(c_int) :: rc
    end function
    !> iogrid(30) / iogrid(31) on host buffers: grid4d = variables3d(4, ix, il, kx), logp(ix, il)
    function sml_dyn_from_grid_host(ctx, grid4d, logp, minmax, safe) bind(C, name='sml_dyn_from_grid_host') &
        result(rc)
      import :: c_ptr, c_double, c_int
      type(c_ptr), value :: ctx
      real(c_double), intent(in) :: grid4d(*), logp(*)
      real(c_double), intent(out) :: minmax(8)
      integer(c_int), intent(out) :: safe
      integer(c_int) :: rc
    end function
    function sml_dyn_to_grid_host(ctx, grid4d, logp) bind(C, name='sml_dyn_to_grid_host') result(rc)
      import :: c_ptr, c_double, c_int
      type(c_ptr), value :: ctx
      real(c_double), intent(out) :: grid4d(*), logp(*)
      integer(c_int) :: rc
    end function

    ! ------------------------------------------------------------ SPEEDY physics / clock
    !> phypar's boundary fields bc(ix*il, 15) (include/speedy_ml.h order); switches the GPU physics on
    function sml_dyn_set_physics(ctx, bc) bind(C, name='sml_dyn_set_physics') result(rc)
      import :: c_ptr, c_double, c_int
      type(c_ptr), value :: ctx
      real(c_double), intent(in) :: bc(*)
      integer(c_int) :: rc
    end function
    !> ini_sea's sea ice (sice_am, tice_am: ngp each; c_null_ptr twice = no ice)
    function sml_dyn_set_sea_ice(ctx, sice, tice) bind(C, name='sml_dyn_set_sea_ice') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx, sice, tice
      integer(c_int) :: rc
    end function
    function sml_dyn_set_rad_state(ctx, rad) bind(C, name='sml_dyn_set_rad_state') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx, rad
      integer(c_int) :: rc
    end function
    function sml_dyn_set_clock(ctx, istep, lradsw) bind(C, name='sml_dyn_set_clock') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int), value :: istep, lradsw
      integer(c_int) :: rc
    end function
    function sml_dyn_get_clock(ctx, istep, lradsw) bind(C, name='sml_dyn_get_clock') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int), intent(out) :: istep, lradsw
      integer(c_int) :: rc
    end function
    !> run_model (mpires.f90:1516-1628) on device grids: iogrid(30) + check, window,
    !> iogrid(31), q floor; an unsafe entry state returns the input grid
    function sml_dyn_run_model(ctx, d_grid4d, d_logp, nleap, delt, alph, rob, wil, d_fc4d, d_fc2d, stream) &
        bind(C, name='sml_dyn_run_model') result(rc)
      import :: c_ptr, c_int, c_double
      type(c_ptr), value :: ctx, d_grid4d, d_logp, d_fc4d, d_fc2d, stream
      integer(c_int), value :: nleap
      real(c_double), value :: delt, alph, rob, wil
      integer(c_int) :: rc
    end function
    !> is_safe_to_run_speedy of the last window entry (waits for its check only)
    function sml_dyn_last_safe(ctx, safe, minmax) bind(C, name='sml_dyn_last_safe') result(rc)
      import :: c_ptr, c_int, c_double
      type(c_ptr), value :: ctx
      integer(c_int), intent(out) :: safe
      real(c_double), intent(out) :: minmax(8)
      integer(c_int) :: rc
    end function

    function sml_dyn_set_check_cus(ctx, first_cu, num_cus) bind(C, name='sml_dyn_set_check_cus') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx
      integer(c_int), value :: first_cu, num_cus
      integer(c_int) :: rc
    end function
    !> give-up time (microseconds) of run_model's exit waiting for the check beside the window
    function sml_dyn_set_check_timeout(ctx, microseconds) bind(C, name='sml_dyn_set_check_timeout') result(rc)
      import :: c_ptr, c_int, c_int64_t
      type(c_ptr), value :: ctx
      integer(c_int64_t), value :: microseconds
      integer(c_int) :: rc
    end function

    ! ------------------------------------------------------------ communicator (RCCL)
    !> startmpi's world (mpires.f90:21-37) for the one collective of the hot path;
    !> the unique id travels through a file rank 0 writes
    function sml_comm_create_file(world, rank, path, timeout_s, comm) bind(C, name='sml_comm_create_file') &
        result(rc)
      import :: c_int, c_char, c_ptr
      integer(c_int), value :: world, rank, timeout_s
      character(kind=c_char), intent(in) :: path(*)
      type(c_ptr), intent(out) :: comm
      integer(c_int) :: rc
    end function
    function sml_comm_rank(comm, world, rank) bind(C, name='sml_comm_rank') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: comm
      integer(c_int), intent(out) :: world, rank
      integer(c_int) :: rc
    end function
    function sml_comm_destroy(comm) bind(C, name='sml_comm_destroy') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: comm
      integer(c_int) :: rc
    end function

    ! ------------------------------------------------------------ the hybrid loop
    function sml_hybrid_create(res, dyn, comm, nleap, delt, alph, rob, wil, overlap, speedy_cus, h) &
        bind(C, name='sml_hybrid_create') result(rc)
      import :: c_ptr, c_int, c_double
      type(c_ptr), value :: res, dyn, comm
      integer(c_int), value :: nleap, overlap, speedy_cus
      real(c_double), value :: delt, alph, rob, wil
      type(c_ptr), intent(out) :: h
      integer(c_int) :: rc
    end function
    function sml_hybrid_destroy(h) bind(C, name='sml_hybrid_destroy') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      integer(c_int) :: rc
    end function
    function sml_hybrid_set_buffers(h, d_feedback, d_local_model, d_outvec, d_grid4d, d_grid2d, d_precip, &
                                    d_fc4d, d_fc2d, d_tisr) bind(C, name='sml_hybrid_set_buffers') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h, d_feedback, d_local_model, d_outvec, d_grid4d, d_grid2d, d_precip, d_fc4d, d_fc2d, &
                            d_tisr
      integer(c_int) :: rc
    end function
    function sml_hybrid_start(h, d_grid4d, d_grid2d, d_precip, d_fc4d, d_fc2d) bind(C, name='sml_hybrid_start') &
        result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h, d_grid4d, d_grid2d, d_precip, d_fc4d, d_fc2d
      integer(c_int) :: rc
    end function
    !> predict -> exchange -> assemble -> run_model -> re-tile (asynchronous)
    function sml_hybrid_step(h) bind(C, name='sml_hybrid_step') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      integer(c_int) :: rc
    end function
    function sml_hybrid_run_speedy(h, run) bind(C, name='sml_hybrid_run_speedy') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      integer(c_int), intent(out) :: run
      integer(c_int) :: rc
    end function
    function sml_hybrid_sync(h) bind(C, name='sml_hybrid_sync') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      integer(c_int) :: rc
    end function
    !> the slab ocean in the loop (before sml_hybrid_set_buffers; exchange rows widen)
    function sml_hybrid_set_slab(h, slab, d_base_sst, d_sea_mask, timestep, timestep_slab, sst_bias) &
        bind(C, name='sml_hybrid_set_slab') result(rc)
      import :: c_ptr, c_int, c_double
      type(c_ptr), value :: h, slab, d_base_sst, d_sea_mask
      integer(c_int), value :: timestep, timestep_slab
      real(c_double), value :: sst_bias
      integer(c_int) :: rc
    end function
    function sml_hybrid_start_slab(h, d_slab_outvec) bind(C, name='sml_hybrid_start_slab') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h, d_slab_outvec
      integer(c_int) :: rc
    end function
    function sml_hybrid_exchange_width(h, width) bind(C, name='sml_hybrid_exchange_width') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      integer(c_int), intent(out) :: width
      integer(c_int) :: rc
    end function
    function sml_hybrid_slab_buffers(h, d_sst_grid, d_ring, ring_len, d_slab_feedback, d_slab_outvec) &
        bind(C, name='sml_hybrid_slab_buffers') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      type(c_ptr), intent(out) :: d_sst_grid, d_ring, d_slab_feedback, d_slab_outvec
      integer(c_int), intent(out) :: ring_len
      integer(c_int) :: rc
    end function
    !> advance from the host's all-gather output d_recv(nout, maxc, world)
    function sml_hybrid_advance_slabs(h, d_recv) bind(C, name='sml_hybrid_advance_slabs') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h, d_recv
      integer(c_int) :: rc
    end function
    !> cross-stream hops: 0 auto, 1 wait-value, 2 events, 3 one-lane signal / wait kernels
    function sml_hybrid_set_hop_mode(h, mode) bind(C, name='sml_hybrid_set_hop_mode') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      integer(c_int), value :: mode
      integer(c_int) :: rc
    end function
    ! each advance also issues the next step's reservoir begin (states one update ahead)
    function sml_hybrid_set_pipelined(h, on) bind(C, name='sml_hybrid_set_pipelined') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      integer(c_int), value :: on
      integer(c_int) :: rc
    end function
    ! a world-1 loop with a transport exchanges through it (ncclAllGather) as at world > 1
    function sml_hybrid_set_force_exchange(h, on) bind(C, name='sml_hybrid_set_force_exchange') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      integer(c_int), value :: on
      integer(c_int) :: rc
    end function
    !> the step's serial chain: 0 auto, 1 the two-stream schedule, 2 on SPEEDY's stream
    function sml_hybrid_set_chain(h, mode) bind(C, name='sml_hybrid_set_chain') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      integer(c_int), value :: mode
      integer(c_int) :: rc
    end function
    function sml_hybrid_chain(h, requested, effective) bind(C, name='sml_hybrid_chain') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      integer(c_int), intent(out) :: requested, effective
      integer(c_int) :: rc
    end function
    function sml_hybrid_exchange_stream(h, stream) bind(C, name='sml_hybrid_exchange_stream') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      type(c_ptr), intent(out) :: stream
      integer(c_int) :: rc
    end function
    function sml_hybrid_exchanges(h, allgathers) bind(C, name='sml_hybrid_exchanges') result(rc)
      import :: c_ptr, c_int, c_int64_t
      type(c_ptr), value :: h
      integer(c_int64_t), intent(out) :: allgathers
      integer(c_int) :: rc
    end function
    function sml_hybrid_hop_mode(h, requested, effective) bind(C, name='sml_hybrid_hop_mode') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: h
      integer(c_int), intent(out) :: requested, effective
      integer(c_int) :: rc
    end function
    !> rank descriptor without a transport (the host moves the slabs)
    function sml_comm_create_local(world, rank, comm) bind(C, name='sml_comm_create_local') result(rc)
      import :: c_ptr, c_int
      integer(c_int), value :: world, rank
      type(c_ptr), intent(out) :: comm
      integer(c_int) :: rc
    end function
    !> the all-gather's layout: maxc, contiguous, perm(numregions) (0-based slab rows)
    function sml_exchange_plan(numregions, world, maxc, contiguous, perm) bind(C, name='sml_exchange_plan') &
        result(rc)
      import :: c_int
      integer(c_int), value :: numregions, world
      integer(c_int), intent(out) :: maxc, contiguous
      integer(c_int), intent(out) :: perm(*)
      integer(c_int) :: rc
    end function

    ! ------------------------------------------------------------ host plumbing
    function sml_device_alloc(bytes, d_ptr) bind(C, name='sml_device_alloc') result(rc)
      import :: c_int64_t, c_ptr, c_int
      integer(c_int64_t), value :: bytes
      type(c_ptr), intent(out) :: d_ptr
      integer(c_int) :: rc
    end function
    function sml_device_free(d_ptr) bind(C, name='sml_device_free') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: d_ptr
      integer(c_int) :: rc
    end function
    function sml_copy_to_device(d_dst, src, bytes) bind(C, name='sml_copy_to_device') result(rc)
      import :: c_ptr, c_int64_t, c_int
      type(c_ptr), value :: d_dst, src
      integer(c_int64_t), value :: bytes
      integer(c_int) :: rc
    end function
    function sml_copy_to_host(dst, d_src, bytes) bind(C, name='sml_copy_to_host') result(rc)
      import :: c_ptr, c_int64_t, c_int
      type(c_ptr), value :: dst, d_src
      integer(c_int64_t), value :: bytes
      integer(c_int) :: rc
    end function
    !> getxyresextent / getoverlapindices (res_domain.f90:123-204), 1-based
    function sml_region_geometry(numregions, region, g) bind(C, name='sml_region_geometry') result(rc)
      import :: c_int
      integer(c_int), value :: numregions, region
      integer(c_int), intent(out) :: g(12)
      integer(c_int) :: rc
    end function
    !> processor_decomposition (res_domain.f90:31-62), 0-based regions
    function sml_processor_decomposition(numregions, numprocs, irank, regions, count) &
        bind(C, name='sml_processor_decomposition') result(rc)
      import :: c_int
      integer(c_int), value :: numregions, numprocs, irank
      integer(c_int), intent(out) :: regions(*), count
      integer(c_int) :: rc
    end function
    !> the window's date-driven forcing (agcm_init, ini_agcm_init.f90:57-89): inbcon's
    !> fmask_l, fmask_s, alb0 (ngp, 3) and the monthly climatologies stl12, snowd12,
    !> soilw12, sst12, sice12 (ngp, 12, 5)
    function sml_dyn_set_surface(ctx, surf) bind(C, name='sml_dyn_set_surface') result(rc)
      import :: c_ptr, c_double, c_int
      type(c_ptr), value :: ctx
      real(c_double), intent(in) :: surf(*)
      integer(c_int) :: rc
    end function
    function sml_dyn_set_climatology(ctx, clim) bind(C, name='sml_dyn_set_climatology') result(rc)
      import :: c_ptr, c_double, c_int
      type(c_ptr), value :: ctx
      real(c_double), intent(in) :: clim(*)
      integer(c_int) :: rc
    end function
    !> newdate(0) + ini_coupler(2) + the hybrid SST + fordate(0) for a window at the date
    function sml_dyn_fordate(ctx, iyear, imonth, iday, stream) bind(C, name='sml_dyn_fordate') result(rc)
      import :: c_ptr, c_int
      type(c_ptr), value :: ctx, stream
      integer(c_int), value :: iyear, imonth, iday
      integer(c_int) :: rc
    end function
    !> run_model's calendar (mpires.f90:1545): the loop refreshes each window's forcing
    function sml_hybrid_set_calendar(h, startyear, hours_base, step_hours) &
        bind(C, name='sml_hybrid_set_calendar') result(rc)
      import :: c_ptr, c_int, c_int64_t
      type(c_ptr), value :: h
      integer(c_int), value :: startyear, step_hours
      integer(c_int64_t), value :: hours_base
      integer(c_int) :: rc
    end function
  end interface

contains

  !> stop with the library's message, like nc_check (mod_io.f90:1732-1744)
  subroutine sml_check(rc, what)
    integer(c_int), intent(in) :: rc
    character(len=*), intent(in) :: what
    character(kind=c_char), pointer :: msg(:)
    integer :: l
    if (rc == SML_OK) return
    call c_f_pointer(sml_last_error(), msg, [1024])
    l = 0
    do while (l < 1024)
      if (msg(l + 1) == c_null_char) exit
      l = l + 1
    end do
    print *, 'libspeedyml error in ', what, ' (', rc, '): ', msg(1:l)
    stop 1
  end subroutine

  !> the dims of a weight file (win_x=n, win_y=ninp, wout_x=nout, wout_y=ncs+n,
  !> rows_x=k, mean_x=36) and its std vector: trained_reservoir_prediction sizes the
  !> reservoir from the file and sets sst_bool_input <=> std(36) > 0.2
  !> (mod_reservoir.f90:1781-1846)
  subroutine sml_weight_file_header(filename, dims, std)
    character(len=*), intent(in) :: filename
    integer(c_int64_t), intent(out) :: dims(6)
    real(c_double), intent(out) :: std(36)
    real(c_float), allocatable, target :: win(:), wout(:), vals(:), mean32(:), std32(:)
    integer(c_int), allocatable, target :: rows(:), cols(:)
    character(kind=c_char, len=len_trim(filename) + 1) :: cpath
    cpath = trim(filename) // c_null_char
    call sml_check(sml_nc_read_region(cpath, dims, c_null_ptr, c_null_ptr, c_null_ptr, c_null_ptr, &
                                      c_null_ptr, c_null_ptr, c_null_ptr), 'sml_nc_read_region(dims)')
    allocate(win(dims(1) * dims(2)), wout(dims(3) * dims(4)), rows(dims(5)), cols(dims(5)), vals(dims(5)))
    allocate(mean32(dims(6)), std32(dims(6)))
    call sml_check(sml_nc_read_region(cpath, dims, c_loc(win), c_loc(wout), c_loc(rows), c_loc(cols), &
                                      c_loc(vals), c_loc(mean32), c_loc(std32)), 'sml_nc_read_region')
    std = real(std32, c_double)
  end subroutine

  !> read_trained_res (mod_io.f90:2911-2956) + the load into the GPU context for
  !> local region i (0-based): the file's fp32 arrays go to the device unchanged.
  subroutine sml_read_trained_res(ctx, i, filename)
    type(c_ptr), intent(in) :: ctx
    integer, intent(in) :: i
    character(len=*), intent(in) :: filename
    integer(c_int64_t) :: dims(6)
    real(c_float), allocatable, target :: win(:), wout(:), vals(:), mean32(:), std32(:)
    integer(c_int), allocatable, target :: rows(:), cols(:)
    real(c_double), allocatable :: mean(:), std(:)
    character(kind=c_char, len=len_trim(filename) + 1) :: cpath
    cpath = trim(filename) // c_null_char
    call sml_check(sml_nc_read_region(cpath, dims, c_null_ptr, c_null_ptr, c_null_ptr, c_null_ptr, &
                                      c_null_ptr, c_null_ptr, c_null_ptr), 'sml_nc_read_region(dims)')
    allocate(win(dims(1) * dims(2)), wout(dims(3) * dims(4)), rows(dims(5)), cols(dims(5)), vals(dims(5)))
    allocate(mean32(dims(6)), std32(dims(6)), mean(dims(6)), std(dims(6)))
    call sml_check(sml_nc_read_region(cpath, dims, c_loc(win), c_loc(wout), c_loc(rows), c_loc(cols), &
                                      c_loc(vals), c_loc(mean32), c_loc(std32)), 'sml_nc_read_region')
    mean = real(mean32, c_double)   ! exact widening, as read_netcdf_1d_dp_opened does
    std = real(std32, c_double)
    call sml_check(sml_res_load_region_f32(ctx, int(i, c_int), rows, cols, vals, win, wout, mean, std), &
                   'sml_res_load_region_f32')
  end subroutine

  !> predict (mod_reservoir.f90:1416) for every local region: packed feedback,
  !> local_model(132, nlocal), outvec(136, nlocal)
  subroutine sml_predict_all(ctx, feedback, local_model, outvec)
    type(c_ptr), intent(in) :: ctx
    real(c_double), intent(in) :: feedback(:), local_model(:, :)
    real(c_double), intent(out) :: outvec(:, :)
    call sml_check(sml_res_step_host(ctx, feedback, local_model, outvec), 'sml_res_step_host')
  end subroutine

end module sml_hip
