!> mpires -- the rank descriptor the reference keeps in its MPI module
!> (src/mpires.f90:1-37: `mpi_res`, filled by startmpi).  On the GPU path the world
!> is the library's RCCL communicator (or a transport-less rank descriptor): one
!> process per GPU, world / rank from sml_comm_rank.  Only `mpi_res` and its set-up
!> live here; the reference module's exchange and SPEEDY driver (sendrecievegrid,
!> run_model, ...) are the native loop's sml_hybrid_* (include/speedy_ml.h).
module mpires
  use iso_c_binding
  use mod_utilities, only: mpi_type
  use sml_hip, only: sml_check, sml_comm_rank
  implicit none

  type(mpi_type) :: mpi_res

contains

  !> startmpi's bookkeeping (:21-37) from a communicator handle (sml_comm_create*)
  subroutine startmpi_from_comm(comm)
    type(c_ptr), intent(in) :: comm
    integer(c_int) :: world, rank
    call sml_check(sml_comm_rank(comm, world, rank), 'sml_comm_rank')
    call set_world(int(world), int(rank))
  end subroutine

  !> the same for a host that knows its world without a communicator
  subroutine set_world(numprocs, proc_num)
    integer, intent(in) :: numprocs, proc_num
    mpi_res%numprocs = numprocs
    mpi_res%proc_num = proc_num
    mpi_res%is_root = proc_num == 0
    mpi_res%is_serial = numprocs == 1
    mpi_res%ierr = 0
    mpi_res%mpi_world = 0
  end subroutine
end module mpires
