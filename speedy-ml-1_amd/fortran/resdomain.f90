!> resdomain -- the domain bookkeeping of src/res_domain.f90 the interface and the
!> host loop need: processor_decomposition (:31-62, the regions of this rank) and
!> initializedomain (:96-121, one reservoir's grid_type extents).  The horizontal
!> extents come from the library's restatement of getxyresextent /
!> getoverlapindices (sml_region_geometry, csrc/sml_internal.hpp); the vertical
!> ones (get_z_res_extent :143-153, getoverlapindices_vert :206-254,
!> get_trainingdataindices(_vert) :256-318) are restated here.
module resdomain
  use iso_c_binding
  use mod_utilities, only: grid_type, model_parameters_type, xgrid, ygrid, zgrid
  use sml_hip, only: sml_check, sml_region_geometry, sml_processor_decomposition
  implicit none

contains

  !> :31-62 -- region_indices / num_of_regions_on_proc of model_parameters%irank
  subroutine processor_decomposition(model_parameters)
    type(model_parameters_type), intent(inout) :: model_parameters
    integer(c_int) :: cnt
    integer(c_int), allocatable :: r(:)
    allocate (r(model_parameters%number_of_regions))
    call sml_check(sml_processor_decomposition(int(model_parameters%number_of_regions, c_int), &
                                               int(model_parameters%numprocs, c_int), &
                                               int(model_parameters%irank, c_int), r, cnt), &
                   'sml_processor_decomposition')
    if (allocated(model_parameters%region_indices)) deallocate (model_parameters%region_indices)
    model_parameters%region_indices = r(1:cnt)
    model_parameters%num_of_regions_on_proc = cnt
  end subroutine

  subroutine initializedomain(num_regions, region_num, overlap, num_vert_levels, vert_level, vert_overlap, grid)
    integer, intent(in) :: num_regions, region_num, overlap, num_vert_levels, vert_level, vert_overlap
    type(grid_type), intent(inout) :: grid
    integer(c_int) :: g(12)
    if (overlap /= 1) stop 'initializedomain: the GPU path is built for overlap = 1 (mod_reservoir.f90:58)'
    call sml_check(sml_region_geometry(int(num_regions, c_int), int(region_num, c_int), g), 'sml_region_geometry')
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
    ! getoverlapindices' flags: x wrap-around, latitude clipped at a pole
    grid%periodicboundary = grid%res_xstart - overlap < 1 .or. grid%res_xend + overlap > xgrid
    grid%pole = grid%res_ystart - overlap < 1 .or. grid%res_yend + overlap > ygrid
    ! get_trainingdataindices: the resolved points inside the input tile
    grid%tdata_xstart = 1 + overlap
    grid%tdata_xend = grid%inputxchunk - overlap
    if (grid%res_ystart - overlap < 1) then
      grid%tdata_ystart = grid%res_ystart
      grid%tdata_yend = grid%inputychunk - overlap
    else if (grid%res_yend + overlap > ygrid) then
      grid%tdata_ystart = 1 + overlap
      grid%tdata_yend = grid%inputychunk - (ygrid - grid%res_yend)
    else
      grid%tdata_ystart = 1 + overlap
      grid%tdata_yend = grid%inputychunk - overlap
    end if
    call z_extents(num_vert_levels, vert_level, vert_overlap, grid)
    grid%overlap = overlap
    grid%num_vert_levels = num_vert_levels
    grid%vert_overlap = vert_overlap
    grid%number_of_regions = num_regions
  end subroutine

  !> the vertical extents of level vert_level of num_vert_levels
  subroutine z_extents(num_vert_levels, vert_level, vert_overlap, grid)
    integer, intent(in) :: num_vert_levels, vert_level, vert_overlap
    type(grid_type), intent(inout) :: grid
    integer :: nz
    nz = zgrid
    grid%reszchunk = nz / num_vert_levels
    grid%res_zstart = (vert_level - 1) * grid%reszchunk + 1
    grid%res_zend = vert_level * grid%reszchunk
    grid%top = grid%res_zstart == 1
    grid%bottom = grid%res_zend == nz
    if (grid%res_zstart - vert_overlap >= 1 .and. grid%res_zend + vert_overlap <= nz) then
      grid%input_zstart = grid%res_zstart - vert_overlap
      grid%input_zend = grid%res_zend + vert_overlap
      grid%inputzchunk = grid%reszchunk + 2 * vert_overlap
    else if (grid%res_zstart - vert_overlap < 1) then
      grid%input_zstart = 1
      grid%input_zend = grid%res_zend + vert_overlap
      grid%inputzchunk = grid%reszchunk + vert_overlap + (grid%res_zstart - 1)
    else
      grid%input_zstart = grid%res_zstart - vert_overlap
      grid%input_zend = nz
      grid%inputzchunk = grid%reszchunk + vert_overlap + (nz - grid%res_zend)
    end if
    if (grid%res_zstart - vert_overlap < 1) then
      grid%tdata_zstart = grid%res_zstart
      grid%tdata_zend = grid%inputzchunk - vert_overlap
    else if (grid%res_zend + vert_overlap > nz) then
      grid%tdata_zstart = 1 + vert_overlap
      grid%tdata_zend = grid%inputzchunk - (nz - grid%res_zend)
    else
      grid%tdata_zstart = 1 + vert_overlap
      grid%tdata_zend = grid%inputzchunk - vert_overlap
    end if
  end subroutine
end module resdomain
