!> sml_hybrid_main -- the Fortran host of the hybrid prediction on the GPU: the
!> reference's parallelmain (src/parallelmain.f90:30-283) with every per-region and
!> per-window routine replaced by the C-ABI of libspeedyml.
!>
!>   startmpi (mpires.f90:21-37)              -> world / rank from the command line,
!>                                               RCCL communicator (sml_comm_create_file)
!>   processor_decomposition (res_domain.f90:31-62)
!>                                            -> sml_processor_decomposition
!>   trained_reservoir_prediction + read_trained_res (mod_reservoir.f90:1781-1884,
!>   mod_io.f90:2911-2956): sizes from the weight file, sst_bool_input <=>
!>   std(36) > 0.2, weights loaded unchanged  -> sml_weight_file_header,
!>                                               sml_read_trained_res
!>   start_prediction (mod_reservoir.f90:938-959): x, feedback, local_model
!>                                            -> saved states + sml_hybrid_start
!>   the time loop (parallelmain.f90:204-270): predict per region, sendrecievegrid
!>   (gather, assemble, run_model, scatter), exit on run_speedy
!>                                            -> sml_hybrid_step, sml_hybrid_run_speedy
!>
!> Inputs under the directory given as the first argument (the reference reads them
!> from its hard-coded /scratch paths):
!>   setup.txt   numregions nsteps nleap overlap speedy_cus / trial_name
!>   weights/worker_XXXX_level_1_<trial_name>.nc       (one per region)
!>   speedy.bin  vor div t ps tr (mod_dynvar, complex), phis tcorh qcorh,
!>               phypar boundary fields bc(ix*il, 15)   (agcm_init's products)
!>   start.bin   analysis grid4d(4,96,48,8) grid2d(96,48) precip(96,48), forecast
!>               grid4d grid2d, tisr(16, numregions), n(numregions) (int32), then
!>               the saved state x of every region in order
!>   slab.bin    (optional: the slab ocean, parallelmain.f90:216-249) timestep,
!>               timestep_slab (int32), base_sst_grid(96,48), sea_mask(96,48),
!>               sice_am(ix*il), tice_am(ix*il), the start sst(4, numregions)
!>               (start_prediction_slab's outvec; unused where a region has no slab),
!>               n(numregions) (int32, 0 = no slab) and each slab state x in order;
!>               with weights/worker_XXXX_ocean_<trial_name>.nc per sst region
!>               (read_trained_ocean_res, mod_io.f90:2958-3007: a region has a slab
!>               reservoir iff its file exists)
!>   forcing.bin (optional: the window's date-driven forcing, agcm_init's coupler and
!>               fordate every window, ini_agcm_init.f90:57-89) fmask_l fmask_s alb0
!>               (ix*il, 3), stl12 snowd12 soilw12 sst12 sice12 (ix*il, 12, 5), the
!>               calendar's start year (int32) and hours before the first step (int64)
!> Output: out_rank<r>.bin = run_speedy(nsteps) as real, then the exchange rows
!> (width, nlocal) (width = 136, or 140 with the slab: outvec + the region's sst),
!> feedback, local_model(132, nlocal), grid4d, grid2d, precip, forecast grid4d,
!> grid2d, x of every local region, and with the slab wholegrid_sst(96,48) and every
!> slab state.
program sml_hybrid_main
  use iso_c_binding
  use sml_hip
  implicit none

  integer, parameter :: ncs = 132, nout = 136, ng4 = 4 * 96 * 48 * 8, ng2 = 96 * 48
  real(c_double), parameter :: rearth = 6.371e+6_c_double, delt = 86400.0_c_double / 96.0_c_double
  real(c_double), parameter :: alph = 0.5_c_double, rob = 0.05_c_double, wil = 0.53_c_double

  character(len=1024) :: dir, arg, trial
  integer :: world, rank, numregions, nsteps, nleap, overlap, speedy_cus, nlocal, i, t, u, nsteps_done
  integer(c_int) :: cnt, run
  integer(c_int), allocatable :: regions(:), nres(:), kres(:), allregions(:)
  integer(c_signed_char), allocatable :: sst(:)
  integer(c_int64_t) :: dims(6)
  integer(c_int64_t), allocatable :: fboff(:)
  real(c_double) :: std(36)
  type(c_ptr) :: res, dyn, comm, hyb
  type(c_ptr) :: d_fb, d_lm, d_ov, d_g4, d_g2, d_pr, d_f4, d_f2, d_tisr, d_a4, d_a2, d_apr, d_b4, d_b2
  complex(c_double_complex), allocatable, target :: vor(:), div(:), tt(:), ps(:), tr(:), phis(:), tcorh(:), qcorh(:)
  real(c_double), allocatable, target :: bc(:), g4(:), g2(:), pr(:), f4(:), f2(:), tisr_all(:, :), tisr(:, :)
  real(c_double), allocatable, target :: x(:), ov(:), fb(:), lm(:), runs(:)
  character(len=:), allocatable :: fname
  ! the date-driven forcing
  logical :: dated
  integer(c_int) :: startyear
  integer(c_int64_t) :: hours_base
  real(c_double), allocatable :: surf(:), clim(:)
  ! slab ocean
  logical :: slab_on
  integer :: nslab, j, width
  logical :: run_exists
  integer(c_int) :: cw, ts, tss
  integer(c_int), allocatable :: slab_ids(:), slab_ninp(:), slab_n(:), slab_k(:), nslab_all(:)
  integer(c_signed_char) :: out_index(4)
  type(c_ptr) :: slab, d_base, d_mask, d_sov, d_sst, d_ring, d_sfb, d_sov2
  real(c_double), allocatable, target :: base(:), smask(:), sice(:), tice(:), sov_all(:, :), sov(:, :), sstg(:)
  integer(c_int) :: ring_len

  call get_command_argument(1, dir)
  world = 1
  rank = 0
  if (command_argument_count() >= 3) then
    call get_command_argument(2, arg)
    read (arg, *) world
    call get_command_argument(3, arg)
    read (arg, *) rank
  end if
  open (newunit=u, file=trim(dir) // '/setup.txt', status='old', action='read')
  read (u, *) numregions, nsteps, nleap, overlap, speedy_cus
  read (u, '(a)') trial
  close (u)

  ! --- startmpi + processor_decomposition
  comm = c_null_ptr
  if (world > 1) call sml_check(sml_comm_create_file(int(world, c_int), int(rank, c_int), &
                                trim(dir) // '/rccl_id' // c_null_char, 120_c_int, comm), 'sml_comm_create_file')
  allocate (regions(numregions))
  call sml_check(sml_processor_decomposition(int(numregions, c_int), int(world, c_int), int(rank, c_int), &
                                             regions, cnt), 'sml_processor_decomposition')
  nlocal = cnt

  ! --- trained_reservoir_prediction: sizes and the sst flag from each region's file
  allocate (nres(nlocal), kres(nlocal), sst(nlocal))
  do i = 1, nlocal
    fname = weight_file(regions(i))
    call sml_weight_file_header(fname, dims, std)
    nres(i) = int(dims(1), c_int)
    kres(i) = int(dims(5), c_int)
    sst(i) = merge(1_c_signed_char, 0_c_signed_char, std(36) > 0.2_c_double)  ! mod_reservoir.f90:1837-1845
  end do
  call sml_check(sml_res_create(int(numregions, c_int), int(nlocal, c_int), regions, sst, nres, kres, &
                                int(ncs, c_int), int(nout, c_int), SML_F32, 1.0_c_double, res), 'sml_res_create')
  do i = 1, nlocal
    call sml_read_trained_res(res, i - 1, weight_file(regions(i)))
  end do

  ! --- trained_ocean_reservoir_prediction (mod_slab_ocean_reservoir.f90:1494-1569):
  ! the slab reservoirs of the rank's regions whose ocean file exists
  inquire (file=trim(dir) // '/slab.bin', exist=slab_on)
  nslab = 0
  if (slab_on) then
    allocate (slab_ids(nlocal), slab_ninp(nlocal), slab_n(nlocal), slab_k(nlocal))
    do i = 1, nlocal
      inquire (file=ocean_file(regions(i)), exist=run_exists)
      if (.not. run_exists) cycle
      nslab = nslab + 1
      call sml_weight_file_header(ocean_file(regions(i)), dims, std)
      slab_ids(nslab) = regions(i)
      slab_n(nslab) = int(dims(1), c_int)
      slab_ninp(nslab) = int(dims(2), c_int)
      slab_k(nslab) = int(dims(5), c_int)
    end do
    out_index = 35_c_signed_char  ! grid%sst_mean_std_idx = 36 (1-based)
    call sml_check(sml_res_create_generic(int(numregions, c_int), int(nslab, c_int), slab_ids, slab_ninp, slab_n, &
                                          slab_k, 0_c_int, 4_c_int, out_index, SML_F32, 1.0_c_double, slab), &
                   'sml_res_create_generic')
    do j = 1, nslab
      call sml_read_trained_res(slab, j - 1, ocean_file(slab_ids(j)))
    end do
  end if

  ! --- SPEEDY: the state and forcing agcm_init leaves, physics boundary fields
  allocate (vor(31 * 32 * 8 * 2), div(31 * 32 * 8 * 2), tt(31 * 32 * 8 * 2), tr(31 * 32 * 8 * 2), ps(31 * 32 * 2))
  allocate (phis(31 * 32), tcorh(31 * 32), qcorh(31 * 32), bc(ng2 * 15))
  open (newunit=u, file=trim(dir) // '/speedy.bin', access='stream', form='unformatted', status='old')
  read (u) vor, div, tt, ps, tr, phis, tcorh, qcorh, bc
  close (u)
  call sml_check(sml_dyn_create(rearth, dyn), 'sml_dyn_create')
  call sml_check(sml_dyn_set_forcing(dyn, phis, tcorh, qcorh), 'sml_dyn_set_forcing')
  call sml_check(sml_dyn_set_state(dyn, vor, div, tt, ps, tr), 'sml_dyn_set_state')
  call sml_check(sml_dyn_set_physics(dyn, bc), 'sml_dyn_set_physics')
  inquire (file=trim(dir) // '/forcing.bin', exist=dated)
  if (dated) then
    allocate (surf(3 * ng2), clim(5 * 12 * ng2))
    open (newunit=u, file=trim(dir) // '/forcing.bin', access='stream', form='unformatted', status='old')
    read (u) surf, clim, startyear, hours_base
    close (u)
    call sml_check(sml_dyn_set_surface(dyn, surf), 'sml_dyn_set_surface')
    call sml_check(sml_dyn_set_climatology(dyn, clim), 'sml_dyn_set_climatology')
  end if

  ! --- start_prediction: saved states, the analysis grid and its SPEEDY forecast
  allocate (g4(ng4), g2(ng2), pr(ng2), f4(ng4), f2(ng2), tisr_all(16, numregions), tisr(16, nlocal))
  allocate (allregions(numregions), fboff(nlocal + 1))
  open (newunit=u, file=trim(dir) // '/start.bin', access='stream', form='unformatted', status='old')
  read (u) g4, g2, pr, f4, f2, tisr_all
  call read_states(u)
  close (u)
  do i = 1, nlocal
    tisr(:, i) = tisr_all(:, regions(i) + 1)
  end do
  call sml_check(sml_res_feedback_offsets(res, fboff), 'sml_res_feedback_offsets')
  d_fb = dalloc(8_c_int64_t * fboff(nlocal + 1))
  d_lm = dalloc(8_c_int64_t * ncs * nlocal)
  d_ov = dalloc(8_c_int64_t * nout * nlocal)
  d_g4 = dalloc(8_c_int64_t * ng4)
  d_g2 = dalloc(8_c_int64_t * ng2)
  d_pr = dalloc(8_c_int64_t * ng2)
  d_f4 = dalloc(8_c_int64_t * ng4)
  d_f2 = dalloc(8_c_int64_t * ng2)
  d_tisr = dalloc(8_c_int64_t * 16 * nlocal)
  d_a4 = dalloc(8_c_int64_t * ng4)
  d_a2 = dalloc(8_c_int64_t * ng2)
  d_apr = dalloc(8_c_int64_t * ng2)
  d_b4 = dalloc(8_c_int64_t * ng4)
  d_b2 = dalloc(8_c_int64_t * ng2)
  call h2d(d_a4, c_loc(g4), ng4)
  call h2d(d_a2, c_loc(g2), ng2)
  call h2d(d_apr, c_loc(pr), ng2)
  call h2d(d_b4, c_loc(f4), ng4)
  call h2d(d_b2, c_loc(f2), ng2)
  call h2d(d_tisr, c_loc(tisr), 16 * nlocal)

  ! --- the loop (parallelmain.f90:204-270)
  call sml_check(sml_hybrid_create(res, dyn, comm, int(nleap, c_int), delt, alph, rob, wil, int(overlap, c_int), &
                                   int(speedy_cus, c_int), hyb), 'sml_hybrid_create')
  if (dated) call sml_check(sml_hybrid_set_calendar(hyb, startyear, hours_base, 6_c_int), 'sml_hybrid_set_calendar')
  if (slab_on) then  ! before the buffers: the exchange rows carry the regions' sst
    allocate (base(ng2), smask(ng2), sice(ng2), tice(ng2), sov_all(4, numregions), nslab_all(numregions))
    open (newunit=u, file=trim(dir) // '/slab.bin', access='stream', form='unformatted', status='old')
    read (u) ts, tss, base, smask, sice, tice, sov_all, nslab_all
    j = 1
    do i = 0, numregions - 1
      if (nslab_all(i + 1) == 0) cycle
      allocate (x(nslab_all(i + 1)))
      read (u) x
      if (j <= nslab) then
        if (slab_ids(j) == i) then
          if (nslab_all(i + 1) /= slab_n(j)) stop 'slab.bin: slab state size differs from the ocean file'
          call sml_check(sml_res_set_state(slab, int(j - 1, c_int), x), 'sml_res_set_state(slab)')
          j = j + 1
        end if
      end if
      deallocate (x)
    end do
    close (u)
    d_base = dalloc(8_c_int64_t * ng2)
    d_mask = dalloc(8_c_int64_t * ng2)
    call h2d(d_base, c_loc(base), ng2)
    call h2d(d_mask, c_loc(smask), ng2)
    call sml_check(sml_dyn_set_sea_ice(dyn, c_loc(sice), c_loc(tice)), 'sml_dyn_set_sea_ice')
    call sml_check(sml_hybrid_set_slab(hyb, slab, d_base, d_mask, ts, tss, 0.0_c_double), 'sml_hybrid_set_slab')
  end if
  call sml_check(sml_hybrid_exchange_width(hyb, cw), 'sml_hybrid_exchange_width')
  width = cw
  call sml_check(sml_device_free(d_ov), 'sml_device_free')
  d_ov = dalloc(8_c_int64_t * width * nlocal)
  call sml_check(sml_hybrid_set_buffers(hyb, d_fb, d_lm, d_ov, d_g4, d_g2, d_pr, d_f4, d_f2, d_tisr), &
                 'sml_hybrid_set_buffers')
  call sml_check(sml_hybrid_start(hyb, d_a4, d_a2, d_apr, d_b4, d_b2), 'sml_hybrid_start')
  if (slab_on) then  ! start_prediction_slab's sst of the slab regions
    allocate (sov(4, max(nslab, 1)))
    do j = 1, nslab
      sov(:, j) = sov_all(:, slab_ids(j) + 1)
    end do
    d_sov = dalloc(8_c_int64_t * 4 * max(nslab, 1))
    call h2d(d_sov, c_loc(sov), 4 * max(nslab, 1))
    call sml_check(sml_hybrid_start_slab(hyb, d_sov), 'sml_hybrid_start_slab')
  end if
  allocate (runs(nsteps))
  runs = -1.0_c_double
  nsteps_done = 0
  do t = 1, nsteps
    call sml_check(sml_hybrid_step(hyb), 'sml_hybrid_step')
    call sml_check(sml_hybrid_run_speedy(hyb, run), 'sml_hybrid_run_speedy')
    runs(t) = real(run, c_double)
    nsteps_done = t
    if (run == 0) exit   ! run_speedy .eqv. .false. (parallelmain.f90:268-270)
  end do
  call sml_check(sml_hybrid_sync(hyb), 'sml_hybrid_sync')
  print '(a,i0,a,i0,a)', 'sml_hybrid_main: rank ', rank, ' ran ', nsteps_done, ' hybrid steps'

  ! --- outputs
  allocate (ov(width * nlocal), fb(fboff(nlocal + 1)), lm(ncs * nlocal))
  call d2h(c_loc(ov), d_ov, width * nlocal)
  call d2h(c_loc(fb), d_fb, int(fboff(nlocal + 1)))
  call d2h(c_loc(lm), d_lm, ncs * nlocal)
  call d2h(c_loc(g4), d_g4, ng4)
  call d2h(c_loc(g2), d_g2, ng2)
  call d2h(c_loc(pr), d_pr, ng2)
  call d2h(c_loc(f4), d_f4, ng4)
  call d2h(c_loc(f2), d_f2, ng2)
  write (arg, '(a,i0,a)') '/out_rank', rank, '.bin'
  open (newunit=u, file=trim(dir) // trim(arg), access='stream', form='unformatted', status='replace')
  write (u) runs, ov, fb, lm, g4, g2, pr, f4, f2
  do i = 1, nlocal
    allocate (x(nres(i)))
    call sml_check(sml_res_get_state(res, i - 1, x), 'sml_res_get_state')
    write (u) x
    deallocate (x)
  end do
  if (slab_on) then
    allocate (sstg(ng2))
    call sml_check(sml_hybrid_slab_buffers(hyb, d_sst, d_ring, ring_len, d_sfb, d_sov2), 'sml_hybrid_slab_buffers')
    call d2h(c_loc(sstg), d_sst, ng2)
    write (u) sstg
    do j = 1, nslab
      allocate (x(slab_n(j)))
      call sml_check(sml_res_get_state(slab, j - 1, x), 'sml_res_get_state(slab)')
      write (u) x
      deallocate (x)
    end do
  end if
  close (u)
  call sml_check(sml_hybrid_destroy(hyb), 'sml_hybrid_destroy')
  call sml_check(sml_dyn_destroy(dyn), 'sml_dyn_destroy')
  call sml_check(sml_res_destroy(res), 'sml_res_destroy')
  if (slab_on) call sml_check(sml_res_destroy(slab), 'sml_res_destroy(slab)')
  if (c_associated(comm)) call sml_check(sml_comm_destroy(comm), 'sml_comm_destroy')
  print '(a)', 'sml_hybrid_main ok'

contains

  !> worker_XXXX_level_1_<trial_name>.nc (read_trained_res, mod_io.f90:2925-2931)
  function weight_file(region) result(f)
    integer(c_int), intent(in) :: region
    character(len=:), allocatable :: f
    character(len=4) :: w
    write (w, '(i0.4)') region
    f = trim(dir) // '/weights/worker_' // w // '_level_1_' // trim(trial) // '.nc'
  end function

  !> worker_XXXX_ocean_<trial_name>.nc (read_trained_ocean_res, mod_io.f90:2974-2977)
  function ocean_file(region) result(f)
    integer(c_int), intent(in) :: region
    character(len=:), allocatable :: f
    character(len=4) :: w
    write (w, '(i0.4)') region
    f = trim(dir) // '/weights/worker_' // w // '_ocean_' // trim(trial) // '.nc'
  end function

  function dalloc(bytes) result(p)
    integer(c_int64_t), intent(in) :: bytes
    type(c_ptr) :: p
    call sml_check(sml_device_alloc(bytes, p), 'sml_device_alloc')
  end function

  subroutine h2d(d, h, n)
    type(c_ptr), intent(in) :: d, h
    integer, intent(in) :: n
    call sml_check(sml_copy_to_device(d, h, 8_c_int64_t * n), 'sml_copy_to_device')
  end subroutine

  subroutine d2h(h, d, n)
    type(c_ptr), intent(in) :: h, d
    integer, intent(in) :: n
    call sml_check(sml_copy_to_host(h, d, 8_c_int64_t * n), 'sml_copy_to_host')
  end subroutine

  !> the saved states of every region: n(numregions) (int32), then each region's x
  !> in region order; the local ones go to the context
  subroutine read_states(unit)
    integer, intent(in) :: unit
    integer :: r, j
    integer(c_int), allocatable :: nall(:)
    real(c_double), allocatable :: xr(:)
    allocate (nall(numregions))
    read (unit) nall
    j = 1
    do r = 0, numregions - 1
      allocate (xr(nall(r + 1)))
      read (unit) xr
      if (j <= nlocal) then
        if (regions(j) == r) then
          if (nall(r + 1) /= nres(j)) stop 'start.bin: state size differs from the weight file'
          call sml_check(sml_res_set_state(res, int(j - 1, c_int), xr), 'sml_res_set_state')
          j = j + 1
        end if
      end if
      deallocate (xr)
    end do
  end subroutine

end program sml_hybrid_main
