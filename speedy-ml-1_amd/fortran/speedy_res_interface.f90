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
!> The derived types are mod_utilities' own (fortran/mod_utilities.f90: the
!> reference's type, component and kind names), and the calendar is mod_calendar's,
!> so the reference's callers compile against this module unchanged.  Like the
!> reference module this one is all public: it re-exports the types it uses.
!> What differs, and why:
!>   * startspeedy does initializedomain(mpi_res%numprocs, mpi_res%proc_num, ...) +
!>     initialize_calendar as the reference (:36-38; mpi_res from module mpires,
!>     which the host fills from its communicator), with vert_level = 1 where the
!>     reference passes an unset local, and when runspeedy is set also creates the
!>     GPU SPEEDY context (speedy_gpu): the device tables that agcm_init rebuilt every
!>     window are built once here.
!>   * test_hybrid_speedy_component starts from internal_state_vector (the
!>     reference reads one ERA-5 file from /scratch, absent here), advances the
!>     calendar and the state's date fields per window as the reference (:778,
!>     :791-800) and runs the window loop through run_model on the GPU
!>     (sml_dyn_run_model) with the reference's clips; hybrid_test_windows (default
!>     500, as the reference's loop) sets its length.  Its netCDF write of each
!>     window is not reproduced, and the date's boundary fields (fordate: the
!>     coupler, out of scope) are the host's, set through sml_dyn_set_physics.
!>   * The ERA / SPEEDY-state readers need the ERA-5 and SPEEDY_STATES netCDF-4
!>     files (parallel HDF5 via MPI-IO) of the reference's /scratch tree; no such
!>     files or library exist on this path, so they stop with a message naming the
!>     file they would open, as nc_check stops on a missing file (mod_io.f90:1732-1744).
!>   * write_restart_new and getspeedyvariable keep the reference's bodies (its
!>     write is commented out; getspeedyvariable prints the step every `stride`;
!>     the step is this module's currentstep, stloop's clock of the GPU context,
!>     where the reference reads mod_tsteps' counter of its CPU SPEEDY).
module speedy_res_interface
  use iso_c_binding, only: c_ptr, c_null_ptr, c_associated, c_int, c_int64_t, c_double, c_loc
  use sml_hip, only: sml_check, sml_dyn_create, sml_dyn_get_clock, sml_device_alloc, sml_device_free, &
                     sml_copy_to_device, sml_copy_to_host, sml_dyn_run_model, sml_dyn_last_safe
  use mod_utilities, only: dp, speedy_data_type, era_data_type, state_vector_type, reservoir_type, grid_type, &
                           model_parameters_type, opened_netcdf_type
  use mod_calendar, only: calendar, initialize_calendar
  implicit none

  ! the binding's names stay inside; everything else is public, as in the reference
  private :: c_ptr, c_null_ptr, c_associated, c_int, c_int64_t, c_double, c_loc
  private :: sml_check, sml_dyn_create, sml_dyn_get_clock, sml_device_alloc, sml_device_free, &
             sml_copy_to_device, sml_copy_to_host, sml_dyn_run_model, sml_dyn_last_safe

  integer, parameter :: numoftimestep = 17, stride = 1, vartime = numoftimestep / stride, &
                        numofspeedyvars = 4, numoflevels = 8

  type(state_vector_type) :: internal_state_vector
  !> the GPU SPEEDY context startspeedy creates (null until then)
  type(c_ptr) :: speedy_gpu = c_null_ptr
  integer :: hybrid_test_windows = 500
  integer :: currentstep = 0

contains

  !> :20-37 -- initializedomain(numprocs, proc_num, overlap, ...) and the calendar;
  !> with runspeedy, the GPU SPEEDY context (tables of indyns / parmtr / inifft)
  subroutine startspeedy(model_parameters, grid, runspeedy)
    use mpires, only: mpi_res
    use resdomain, only: initializedomain
    type(model_parameters_type), intent(in) :: model_parameters
    type(grid_type), intent(inout) :: grid
    logical, intent(in) :: runspeedy
    integer :: vert_level
    vert_level = 1
    call initializedomain(mpi_res%numprocs, mpi_res%proc_num, model_parameters%overlap, grid%num_vert_levels, &
                          vert_level, grid%vert_overlap, grid)
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
    if (.false.) print *, reservoir%n, grid%number_of_regions, model_parameters%irank, end_year, allocated(era_data%era_logp), &
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
    if (.false.) print *, reservoir%n, grid%number_of_regions, model_parameters%irank, end_year, allocated(era_data%era_logp), &
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
    if (.false.) print *, reservoir%n, grid%number_of_regions, model_parameters%irank, end_year, &
                          allocated(speedy_data%speedy_logp), present(timestep_arg)
    call missing_input('read_model_states', '/scratch/user/troyarcomano/SPEEDY_STATES/restart_6hour_y' // year // '.nc')
  end subroutine

  !> :722-815 -- repeated SPEEDY windows from internal_state_vector: the calendar
  !> advanced to hour 86184 + i and the state's start / date fields set from it
  !> (:778, :789-800), q clipped to [0, 25] before each window, run_model (here
  !> sml_dyn_run_model: iogrid(30), stepone + 24 leapfrog steps, iogrid(31), q floor
  !> 1e-6), q < 0 -> 0 after.
  !> The GPU context must have its state, forcing and physics set (startspeedy
  !> creates it).  Stops early when a window is unsafe (is_safe_to_run_speedy).
  subroutine test_hybrid_speedy_component()
    use mod_calendar, only: get_current_time_delta_hour
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
      call get_current_time_delta_hour(calendar, 86184 + i)
      where (internal_state_vector%variables3d(4, :, :, :) < 0.0_dp) internal_state_vector%variables3d(4, :, :, :) = 0.0_dp
      where (internal_state_vector%variables3d(4, :, :, :) > 25.0_dp) &
        internal_state_vector%variables3d(4, :, :, :) = 25.0_dp
      internal_state_vector%is_safe_to_run_speedy = .true.
      internal_state_vector%era_hour = 1
      internal_state_vector%era_hour_plus_one = 2
      internal_state_vector%istart = 2
      internal_state_vector%era_start = 3
      internal_state_vector%iyear0 = calendar%currentyear
      internal_state_vector%imont0 = calendar%currentmonth
      internal_state_vector%iday = calendar%currentday
      internal_state_vector%ihour = calendar%currenthour
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
