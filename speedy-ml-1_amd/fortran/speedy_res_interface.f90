!> speedy_res_interface -- the reference's ML<->SPEEDY interface module
!> (src/speedy_res_interface.f90:1-838), same module name, same public names and
!> argument lists, over the GPU path:
!>
!>   startspeedy(model_parameters, grid, runspeedy)        :20-37
!>   write_restart_new(filename, timestep, grid4d, grid2d) :51-61
!>   getspeedyvariable()                                   :63-91
!>   read_era_netcdf_opened(reservoir, grid, model_parameters, start_year, end_year,
!>                          era_data, netcdf_files, timestep_arg)   :248-437
!>   read_era(reservoir, grid, model_parameters, start_year, end_year, era_data,
!>            timestep_arg)                                :439-632
!>   read_model_states(reservoir, grid, model_parameters, start_year, end_year,
!>                     speedy_data, timestep_arg)          :634-720
!>   test_hybrid_speedy_component()                        :722-815
!>   truncate_letkf_code_version(field_orig, trunc_twn)    :817-837
!>   internal_state_vector (module variable)               :17
!>
!> The derived types are the subsets of mod_utilities' types these routines touch
!> (mod_utilities.f90:32-604).  What differs, and why:
!>   * startspeedy does initializedomain + initialize_calendar as the reference, and
!>     when runspeedy is set also creates the GPU SPEEDY context (speedy_gpu): the
!>     device tables that agcm_init rebuilt every window are built once here.
!>   * test_hybrid_speedy_component starts from internal_state_vector (the
!>     reference reads one ERA-5 file from /scratch, absent here) and runs the
!>     window loop through run_model on the GPU (sml_dyn_run_model) with the
!>     reference's clips; hybrid_test_windows (default 500, as the reference's loop)
!>     sets its length.  Its netCDF write of each window is not reproduced.
!>   * The ERA / SPEEDY-state readers need the ERA-5 and SPEEDY_STATES netCDF-4
!>     files (parallel HDF5 via MPI-IO) of the reference's /scratch tree; no such
!>     files or library exist on this path, so they stop with a message naming the
!>     file they would open, as nc_check stops on a missing file (mod_io.f90:1732-1744).
!>   * write_restart_new and getspeedyvariable keep the reference's bodies (its
!>     write is commented out; getspeedyvariable prints the step every `stride`).
module speedy_res_interface
  use iso_c_binding
  use sml_hip
  implicit none
  private

  integer, parameter, public :: dp = kind(1.d0)
  integer, parameter, public :: numoftimestep = 17, stride = 1, vartime = numoftimestep / stride, &
                                numofspeedyvars = 4, numoflevels = 8

  !> subsets of mod_utilities.f90's types (field names as there)
  type, public :: model_parameters_type
    integer :: number_of_regions = 1152, num_of_regions_on_proc = 0, irank = 0, numprocs = 1
    integer :: overlap = 1, num_vert_levels = 1, vert_loc_overlap = 0, timestep = 6
    integer :: chunk_size_prediction = 136, chunk_size_speedy = 132
    integer, allocatable :: region_indices(:)
    logical :: run_speedy = .true., ml_only = .false., slab_ocean_model_bool = .false.
    character(len=:), allocatable :: trial_name
  end type

  type, public :: grid_type
    integer :: res_xstart, res_xend, res_ystart, res_yend, resxchunk, resychunk
    integer :: input_xstart, input_xend, input_ystart, input_yend, inputxchunk, inputychunk
    integer :: reszchunk = 8, inputzchunk = 8, res_zstart = 1, res_zend = 8, input_zstart = 1, input_zend = 8
    integer :: num_vert_levels = 1, level_index = 1, vert_overlap = 0, number_of_regions = 1152, region = 0
    logical :: pole = .false., periodicboundary = .false.
    real(dp), allocatable :: mean(:), std(:)
  end type

  type, public :: reservoir_type
    integer :: assigned_region = -1, n = 0, k = 0, reservoir_numinputs = 0
    logical :: sst_bool = .false., sst_climo_bool = .false., tisr_input_bool = .true., precip_bool = .true.
  end type

  type, public :: state_vector_type
    real(dp), allocatable :: variables3d(:, :, :, :), logp(:, :), sst_hybrid(:, :)
    integer :: istart = 2, era_start = 3, era_hour = 1, era_hour_plus_one = 2
    integer :: iyear0 = 1981, imont0 = 1, iday = 1, ihour = 0
    logical :: is_safe_to_run_speedy = .true., hybrid_slab = .false.
    real(dp) :: sst_bias = 0.0_dp
  end type

  type, public :: speedy_data_type
    real(dp), allocatable :: speedyvariables(:, :, :, :, :), speedy_logp(:, :, :)
  end type

  type, public :: era_data_type
    real(dp), allocatable :: eravariables(:, :, :, :, :), era_logp(:, :, :), era_tisr(:, :, :), &
                             era_sst(:, :, :), era_sst_climo(:, :, :), era_precip(:, :, :)
  end type

  type, public :: opened_netcdf_type
    character(len=:), allocatable :: filename
    logical :: is_opened = .false.
    integer :: ncid = -1
  end type

  !> mod_calendar's calendar (initialize_calendar(calendar, 1981, 1, 1, 0))
  type, public :: calendar_type
    integer :: startyear, startmonth, startday, starthour
    integer :: currentyear, currentmonth, currentday, currenthour
  end type

  type(state_vector_type), public :: internal_state_vector
  type(calendar_type), public :: calendar
  !> the GPU SPEEDY context startspeedy creates (null until then)
  type(c_ptr), public :: speedy_gpu = c_null_ptr
  integer, public :: hybrid_test_windows = 500
  integer, public :: currentstep = 0

  public :: startspeedy, write_restart_new, getspeedyvariable, read_era_netcdf_opened, read_era, &
            read_model_states, test_hybrid_speedy_component, truncate_letkf_code_version, initializedomain, &
            initialize_calendar

contains

  !> initializedomain (res_domain.f90:96-121): the region's extent and its overlap
  !> input extent (getxyresextent / getoverlapindices, :123-204)
  subroutine initializedomain(numregions, region, overlap, num_vert_levels, vert_level, vert_overlap, grid)
    integer, intent(in) :: numregions, region, overlap, num_vert_levels, vert_level, vert_overlap
    type(grid_type), intent(inout) :: grid
    integer(c_int) :: g(12)
    if (overlap /= 1) stop 'initializedomain: the GPU path is built for overlap = 1 (mod_reservoir.f90:58)'
    call sml_check(sml_region_geometry(int(numregions, c_int), int(region, c_int), g), 'sml_region_geometry')
    grid%number_of_regions = numregions
    grid%region = region
    grid%res_xstart = g(1)
    grid%res_xend = g(2)
    grid%res_ystart = g(3)
    grid%res_yend = g(4)
    grid%resxchunk = g(5)
    grid%resychunk = g(6)
    grid%input_xstart = g(7)
    grid%input_xend = g(8)
    grid%input_ystart = g(9)
    grid%input_yend = g(10)
    grid%inputxchunk = g(11)
    grid%inputychunk = g(12)
    grid%pole = grid%res_ystart == 1 .or. grid%res_yend == 48
    grid%periodicboundary = grid%input_xstart > grid%res_xstart .or. grid%input_xend < grid%res_xend
    grid%num_vert_levels = num_vert_levels
    grid%level_index = vert_level
    grid%vert_overlap = vert_overlap
  end subroutine

  subroutine initialize_calendar(cal, year, month, day, hour)
    type(calendar_type), intent(inout) :: cal
    integer, intent(in) :: year, month, day, hour
    cal%startyear = year
    cal%startmonth = month
    cal%startday = day
    cal%starthour = hour
    cal%currentyear = year
    cal%currentmonth = month
    cal%currentday = day
    cal%currenthour = hour
  end subroutine

  !> :20-37 -- initializedomain(numprocs, proc_num, overlap, ...) and the calendar;
  !> with runspeedy, the GPU SPEEDY context (tables of indyns / parmtr / inifft)
  subroutine startspeedy(model_parameters, grid, runspeedy)
    type(model_parameters_type), intent(in) :: model_parameters
    type(grid_type), intent(inout) :: grid
    logical, intent(in) :: runspeedy
    integer :: vert_level
    vert_level = 1
    call initializedomain(model_parameters%number_of_regions, model_parameters%irank, model_parameters%overlap, &
                          grid%num_vert_levels, vert_level, grid%vert_overlap, grid)
    call initialize_calendar(calendar, 1981, 1, 1, 0)
    if (runspeedy .and. .not. c_associated(speedy_gpu)) &
      call sml_check(sml_dyn_create(6.371e+6_c_double, speedy_gpu), 'sml_dyn_create')
  end subroutine

  !> :51-61 -- the reference's body is commented out (write_netcdf_speedy_full_mpi)
  subroutine write_restart_new(filename, timestep, grid4d, grid2d)
    character(len=*), intent(in) :: filename
    integer, intent(in) :: timestep
    real(kind=dp), intent(in) :: grid4d(:, :, :, :)
    real(kind=dp), intent(in) :: grid2d(:, :)
    if (.false.) print *, filename, timestep, size(grid4d), size(grid2d)
  end subroutine

  !> :63-91 -- prints the step every `stride` steps (the copies into speedy_data are
  !> commented out in the reference); the step is stloop's clock of the GPU context
  subroutine getspeedyvariable()
    integer(c_int) :: istep, lradsw
    if (c_associated(speedy_gpu)) then
      call sml_check(sml_dyn_get_clock(speedy_gpu, istep, lradsw), 'sml_dyn_get_clock')
      currentstep = istep
    end if
    if (mod(currentstep, stride) == 0) print *, currentstep, 'step'
  end subroutine

  subroutine missing_input(what, path)
    character(len=*), intent(in) :: what, path
    print *, trim(what), ': the reference reads ', trim(path), &
             ' (netCDF-4 / MPI-IO, reference /scratch tree); not available on this path'
    stop 1
  end subroutine

  !> :248-437 -- ERA-5 training data of the region, years start_year..end_year
  subroutine read_era_netcdf_opened(reservoir, grid, model_parameters, start_year, end_year, era_data, &
                                    netcdf_files, timestep_arg)
    type(reservoir_type), intent(inout) :: reservoir
    type(grid_type), intent(inout) :: grid
    type(model_parameters_type), intent(in) :: model_parameters
    integer, intent(in) :: start_year, end_year
    type(era_data_type), intent(inout) :: era_data
    type(opened_netcdf_type), intent(inout) :: netcdf_files(:)
    integer, intent(in), optional :: timestep_arg
    character(len=4) :: year
    write (year, '(i4)') start_year
    if (.false.) print *, reservoir%n, grid%region, model_parameters%irank, end_year, allocated(era_data%era_logp), &
                          size(netcdf_files), present(timestep_arg)
    call missing_input('read_era_netcdf_opened', '/scratch/user/troyarcomano/ERA_5/' // year // '/era_5_y' // year // &
                       '_regridded_mpi_fixed_var_gcc.nc')
  end subroutine

  !> :439-632
  subroutine read_era(reservoir, grid, model_parameters, start_year, end_year, era_data, timestep_arg)
    type(reservoir_type), intent(inout) :: reservoir
    type(grid_type), intent(inout) :: grid
    type(model_parameters_type), intent(in) :: model_parameters
    integer, intent(in) :: start_year, end_year
    type(era_data_type), intent(inout) :: era_data
    integer, intent(in), optional :: timestep_arg
    character(len=4) :: year
    write (year, '(i4)') start_year
    if (.false.) print *, reservoir%n, grid%region, model_parameters%irank, end_year, allocated(era_data%era_logp), &
                          present(timestep_arg)
    call missing_input('read_era', '/scratch/user/troyarcomano/ERA_5/' // year // '/era_5_y' // year // &
                       '_regridded_mpi_fixed_var_gcc.nc')
  end subroutine

  !> :634-720
  subroutine read_model_states(reservoir, grid, model_parameters, start_year, end_year, speedy_data, timestep_arg)
    type(reservoir_type), intent(inout) :: reservoir
    type(grid_type), intent(inout) :: grid
    type(model_parameters_type), intent(in) :: model_parameters
    integer, intent(in) :: start_year, end_year
    type(speedy_data_type), intent(inout) :: speedy_data
    integer, intent(in), optional :: timestep_arg
    character(len=4) :: year
    write (year, '(i4)') start_year
    if (.false.) print *, reservoir%n, grid%region, model_parameters%irank, end_year, &
                          allocated(speedy_data%speedy_logp), present(timestep_arg)
    call missing_input('read_model_states', '/scratch/user/troyarcomano/SPEEDY_STATES/restart_6hour_y' // year // '.nc')
  end subroutine

  !> :722-815 -- repeated SPEEDY windows from internal_state_vector: q clipped to
  !> [0, 25] before each window, run_model (here sml_dyn_run_model: iogrid(30),
  !> stepone + 24 leapfrog steps, iogrid(31), q floor 1e-6), q < 0 -> 0 after.
  !> The GPU context must have its state, forcing and physics set (startspeedy
  !> creates it).  Stops early when a window is unsafe (is_safe_to_run_speedy).
  subroutine test_hybrid_speedy_component()
    integer, parameter :: ng4 = 4 * 96 * 48 * 8, ng2 = 96 * 48
    type(c_ptr) :: d_in4, d_in2, d_out4, d_out2
    integer :: i
    integer(c_int) :: safe
    real(c_double) :: mm(8)
    real(dp), allocatable, target :: v4(:, :, :, :), lp(:, :)
    if (.not. c_associated(speedy_gpu)) stop 'test_hybrid_speedy_component: call startspeedy(..., .true.) first'
    if (.not. allocated(internal_state_vector%variables3d)) allocate (internal_state_vector%variables3d(4, 96, 48, 8))
    if (.not. allocated(internal_state_vector%logp)) allocate (internal_state_vector%logp(96, 48))
    allocate (v4(4, 96, 48, 8), lp(96, 48))
    call sml_check(sml_device_alloc(8_c_int64_t * ng4, d_in4), 'sml_device_alloc')
    call sml_check(sml_device_alloc(8_c_int64_t * ng2, d_in2), 'sml_device_alloc')
    call sml_check(sml_device_alloc(8_c_int64_t * ng4, d_out4), 'sml_device_alloc')
    call sml_check(sml_device_alloc(8_c_int64_t * ng2, d_out2), 'sml_device_alloc')
    do i = 1, hybrid_test_windows
      where (internal_state_vector%variables3d(4, :, :, :) < 0.0_dp) internal_state_vector%variables3d(4, :, :, :) = 0.0_dp
      where (internal_state_vector%variables3d(4, :, :, :) > 25.0_dp) &
        internal_state_vector%variables3d(4, :, :, :) = 25.0_dp
      internal_state_vector%is_safe_to_run_speedy = .true.
      v4 = internal_state_vector%variables3d
      lp = internal_state_vector%logp
      call sml_check(sml_copy_to_device(d_in4, c_loc(v4), 8_c_int64_t * ng4), 'sml_copy_to_device')
      call sml_check(sml_copy_to_device(d_in2, c_loc(lp), 8_c_int64_t * ng2), 'sml_copy_to_device')
      call sml_check(sml_dyn_run_model(speedy_gpu, d_in4, d_in2, 24_c_int, 900.0_c_double, 0.5_c_double, &
                                       0.05_c_double, 0.53_c_double, d_out4, d_out2, c_null_ptr), 'sml_dyn_run_model')
      call sml_check(sml_dyn_last_safe(speedy_gpu, safe, mm), 'sml_dyn_last_safe')
      internal_state_vector%is_safe_to_run_speedy = safe /= 0
      call sml_check(sml_copy_to_host(c_loc(v4), d_out4, 8_c_int64_t * ng4), 'sml_copy_to_host')
      call sml_check(sml_copy_to_host(c_loc(lp), d_out2, 8_c_int64_t * ng2), 'sml_copy_to_host')
      internal_state_vector%variables3d = v4
      internal_state_vector%logp = lp
      print *, 'after speedy specific humidity', minval(internal_state_vector%variables3d(4, :, :, :)), &
               maxval(internal_state_vector%variables3d(4, :, :, :))
      where (internal_state_vector%variables3d(4, :, :, :) < 0.0_dp) internal_state_vector%variables3d(4, :, :, :) = 0.0_dp
      if (.not. internal_state_vector%is_safe_to_run_speedy) exit
    end do
    call sml_check(sml_device_free(d_in4), 'sml_device_free')
    call sml_check(sml_device_free(d_in2), 'sml_device_free')
    call sml_check(sml_device_free(d_out4), 'sml_device_free')
    call sml_check(sml_device_free(d_out2), 'sml_device_free')
  end subroutine

  !> :817-837 -- zero every coefficient with (m-1) + (n-1) > trunc_twn
  function truncate_letkf_code_version(field_orig, trunc_twn) result(field_new)
    complex(dp), intent(in) :: field_orig(:, :)
    integer, intent(in) :: trunc_twn
    complex(dp), allocatable :: field_new(:, :)
    integer :: mx_lr, nx_lr, m, n
    allocate (field_new, mold=field_orig)
    mx_lr = size(field_orig, 1)
    nx_lr = size(field_orig, 2)
    do m = 1, mx_lr
      do n = 1, nx_lr
        field_new(m, n) = field_orig(m, n)
        if (m + n - 2 > trunc_twn) field_new(m, n) = (0.0_dp, 0.0_dp)
      end do
    end do
  end function

end module speedy_res_interface
