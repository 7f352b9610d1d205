!> sml_interface_check -- drives speedy_res_interface (the reference's module names
!> and signatures) on the GPU path; used by tests/test_fortran_hybrid_gpu.py.
!> Reads from the directory in argument 1:
!>   speedy.bin  (as sml_hybrid_main) -- the GPU SPEEDY context's state, forcing, physics
!>   iface_in.bin  variables3d(4,96,48,8), logp(96,48), nwin (int32), trunc_twn (int32),
!>                 field(31,32) complex, nreg (int32), regions(nreg) (int32)
!> Writes iface_out.bin: the internal_state_vector after test_hybrid_speedy_component
!> (variables3d, logp, is_safe as real), truncate_letkf_code_version(field), and per
!> region the 12 startspeedy grid extents (as real).
program sml_interface_check
  use iso_c_binding
  use sml_hip
  use speedy_res_interface
  use mpires, only: set_world
  implicit none
  character(len=1024) :: dir
  integer :: u, i, j
  integer(c_int) :: nwin, trunc_twn, nreg
  integer(c_int), allocatable :: regions(:)
  complex(c_double_complex), allocatable, target :: vor(:), div(:), tt(:), ps(:), tr(:), phis(:), tcorh(:), qcorh(:)
  real(c_double), allocatable, target :: bc(:)
  complex(dp) :: field(31, 32)
  complex(dp), allocatable :: tfield(:, :)
  type(model_parameters_type) :: mp
  type(grid_type) :: grid
  real(dp), allocatable :: ext(:, :)

  call get_command_argument(1, dir)
  mp%number_of_regions = 1152
  mp%overlap = 1
  grid%num_vert_levels = 1
  grid%vert_overlap = 0
  ! the reference's startspeedy decomposes by the MPI world: with 1152 ranks, rank r
  ! gets region r's extents (speedy_res_interface.f90:36)
  call set_world(1152, 0)
  call startspeedy(mp, grid, .true.)   ! region 0 (rank 0), GPU SPEEDY context
  allocate (vor(31 * 32 * 16), div(31 * 32 * 16), tt(31 * 32 * 16), tr(31 * 32 * 16), ps(31 * 32 * 2))
  allocate (phis(31 * 32), tcorh(31 * 32), qcorh(31 * 32), bc(4608 * 15))
  open (newunit=u, file=trim(dir) // '/speedy.bin', access='stream', form='unformatted', status='old')
  read (u) vor, div, tt, ps, tr, phis, tcorh, qcorh, bc
  close (u)
  call sml_check(sml_dyn_set_forcing(speedy_gpu, phis, tcorh, qcorh), 'sml_dyn_set_forcing')
  call sml_check(sml_dyn_set_state(speedy_gpu, vor, div, tt, ps, tr), 'sml_dyn_set_state')
  call sml_check(sml_dyn_set_physics(speedy_gpu, bc), 'sml_dyn_set_physics')

  allocate (internal_state_vector%variables3d(4, 96, 48, 8), internal_state_vector%logp(96, 48))
  open (newunit=u, file=trim(dir) // '/iface_in.bin', access='stream', form='unformatted', status='old')
  read (u) internal_state_vector%variables3d, internal_state_vector%logp, nwin, trunc_twn, field, nreg
  allocate (regions(nreg))
  read (u) regions
  close (u)
  hybrid_test_windows = nwin
  call test_hybrid_speedy_component()
  call getspeedyvariable()
  tfield = truncate_letkf_code_version(field, int(trunc_twn))
  allocate (ext(12, nreg))
  do i = 1, nreg
    call set_world(1152, int(regions(i)))
    call startspeedy(mp, grid, .false.)
    ext(:, i) = real([grid%res_xstart, grid%res_xend, grid%res_ystart, grid%res_yend, grid%resxchunk, &
                      grid%resychunk, grid%input_xstart, grid%input_xend, grid%input_ystart, grid%input_yend, &
                      grid%inputxchunk, grid%inputychunk], dp)
  end do
  open (newunit=u, file=trim(dir) // '/iface_out.bin', access='stream', form='unformatted', status='replace')
  write (u) internal_state_vector%variables3d, internal_state_vector%logp, &
            merge(1.0_dp, 0.0_dp, internal_state_vector%is_safe_to_run_speedy), tfield, ext
  close (u)
  j = calendar%currentyear
  print '(a,i0)', 'sml_interface_check ok, calendar year ', j
  print '(a,4(1x,i0),a,4(1x,i0))', 'calendar', calendar%currentyear, calendar%currentmonth, calendar%currentday, &
    calendar%currenthour, ' state', internal_state_vector%iyear0, internal_state_vector%imont0, &
    internal_state_vector%iday, internal_state_vector%ihour
end program
