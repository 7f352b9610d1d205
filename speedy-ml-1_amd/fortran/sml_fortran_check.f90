!> sml_fortran_check -- a Fortran host driving the GPU path through sml_hip, the
!> way the reference's parallelmain would: read the per-region trained weight files
!> (read_trained_res), load them, set the states, predict all local regions, and
!> transform spectral fields with grid/spec.  Used by tests/test_fortran_gpu.py.
!>
!> usage: sml_fortran_check <dir>
!>   <dir>/inputs.bin  (stream): nlocal, nf, ids(nlocal), sst(nlocal), n(nlocal),
!>                     k(nlocal), feedback(sum ninp), local_model(132,nlocal),
!>                     x0(sum n), spec(62,32,nf), grid(96,48,nf)
!>   <dir>/worker_XXXX.nc per region
!>   writes <dir>/outputs.bin: outvec(136,nlocal), x1(sum n), grid_of_spec(96,48,nf),
!>                     spec_of_grid(62,32,nf)
program sml_fortran_check
  use iso_c_binding
  use sml_hip
  implicit none
  character(len=512) :: dir
  character(len=600) :: fname
  integer(c_int) :: nlocal, nf, i, off, ntot, nfb
  integer(c_int), allocatable :: ids(:), n(:), k(:)
  integer(c_signed_char), allocatable :: sst(:)
  integer(c_int64_t), allocatable :: fboff(:)
  real(c_double), allocatable :: feedback(:), local_model(:, :), x0(:), x1(:), outvec(:, :)
  real(c_double), allocatable :: spec(:, :, :), grid(:, :, :), grid_out(:, :, :), spec_out(:, :, :)
  type(c_ptr) :: res, sp

  call get_command_argument(1, dir)
  open(unit=10, file=trim(dir)//'/inputs.bin', access='stream', form='unformatted', status='old')
  read(10) nlocal, nf
  allocate(ids(nlocal), sst(nlocal), n(nlocal), k(nlocal))
  read(10) ids, sst, n, k
  ntot = sum(n)

  call sml_check(sml_res_create(1152_c_int, nlocal, ids, sst, n, k, 132_c_int, 136_c_int, SML_F32, 1.0_c_double, &
                                res), 'sml_res_create')
  allocate(fboff(nlocal + 1))
  call sml_check(sml_res_feedback_offsets(res, fboff), 'sml_res_feedback_offsets')
  nfb = int(fboff(nlocal + 1))
  allocate(feedback(nfb), local_model(132, nlocal), x0(ntot), x1(ntot), outvec(136, nlocal))
  allocate(spec(62, 32, nf), grid(96, 48, nf), grid_out(96, 48, nf), spec_out(62, 32, nf))
  read(10) feedback, local_model, x0, spec, grid
  close(10)

  off = 0
  do i = 1, nlocal
    write(fname, '(a,"/worker_",i4.4,".nc")') trim(dir), ids(i)
    call sml_read_trained_res(res, i - 1, trim(fname))
    call sml_check(sml_res_set_state(res, i - 1, x0(off + 1:off + n(i))), 'sml_res_set_state')
    off = off + n(i)
  end do

  call sml_predict_all(res, feedback, local_model, outvec)

  off = 0
  do i = 1, nlocal
    call sml_check(sml_res_get_state(res, i - 1, x1(off + 1:off + n(i))), 'sml_res_get_state')
    off = off + n(i)
  end do

  call sml_check(sml_spectral_create(6.371e6_c_double, sp), 'sml_spectral_create')
  call sml_check(sml_grid_host(sp, spec, grid_out, nf, 1_c_int), 'sml_grid_host')
  call sml_check(sml_spec_host(sp, grid, spec_out, nf), 'sml_spec_host')

  open(unit=11, file=trim(dir)//'/outputs.bin', access='stream', form='unformatted', status='replace')
  write(11) outvec, x1, grid_out, spec_out
  close(11)
  call sml_check(sml_spectral_destroy(sp), 'destroy')
  call sml_check(sml_res_destroy(res), 'destroy')
  print *, 'sml_fortran_check ok: regions', nlocal, ' fields', nf, ' abi', sml_abi_version()
end program
