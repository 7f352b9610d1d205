!> sml_dropin_check -- the reference's spectral call sites, unchanged in form
!> (implicit-interface `call grid(vorm, vorg, kcos)` etc., as dyn_grtend.f90,
!> phy_phypar.f90 and ppo_iogrid.f90 make them), resolved at link time by
!> libspeedyml_dropin.so instead of spe_spectral.o / spe_subfft_fftpack.o.
!> Reads dropin_in.bin (nf, spec_in(62,32,nf), grid_in(96,48,nf), grid_in2(96,48,nf))
!> from the directory in argument 1 and writes dropin_out.bin:
!>   grid k1, grid k2 (96,48,nf each), spec (62,32,nf), gridy (62,48,nf),
!>   specy(gridy) (62,32,nf), specx (62,48,nf), vdspec k1 vor/div, k2 vor/div,
!>   uvspec u/v (62,32,nf each)
program sml_dropin_check
  implicit none
  integer, parameter :: dp = kind(1.d0)
  character(len=1024) :: dir
  integer :: nf, f, u
  real(dp), allocatable :: spec_in(:, :, :), grid_in(:, :, :), grid_in2(:, :, :)
  real(dp), allocatable :: gk1(:, :, :), gk2(:, :, :), sp(:, :, :), gy(:, :, :), sy(:, :, :), sx(:, :, :)
  real(dp), allocatable :: v1(:, :, :), d1(:, :, :), v2(:, :, :), d2(:, :, :), uu(:, :, :), vv(:, :, :)

  call get_command_argument(1, dir)
  open (newunit=u, file=trim(dir) // '/dropin_in.bin', access='stream', form='unformatted', status='old')
  read (u) nf
  allocate (spec_in(62, 32, nf), grid_in(96, 48, nf), grid_in2(96, 48, nf))
  read (u) spec_in, grid_in, grid_in2
  close (u)
  allocate (gk1(96, 48, nf), gk2(96, 48, nf), sp(62, 32, nf), gy(62, 48, nf), sy(62, 32, nf), sx(62, 48, nf))
  allocate (v1(62, 32, nf), d1(62, 32, nf), v2(62, 32, nf), d2(62, 32, nf), uu(62, 32, nf), vv(62, 32, nf))
  do f = 1, nf
    call grid(spec_in(1, 1, f), gk1(1, 1, f), 1)
    call grid(spec_in(1, 1, f), gk2(1, 1, f), 2)
    call spec(grid_in(1, 1, f), sp(1, 1, f))
    call gridy(spec_in(1, 1, f), gy(1, 1, f))
    call specy(gy(1, 1, f), sy(1, 1, f))
    call specx(grid_in(1, 1, f), sx(1, 1, f))
    call vdspec(grid_in(1, 1, f), grid_in2(1, 1, f), v1(1, 1, f), d1(1, 1, f), 1)
    call vdspec(grid_in(1, 1, f), grid_in2(1, 1, f), v2(1, 1, f), d2(1, 1, f), 2)
    call uvspec(spec_in(1, 1, f), spec_in(1, 1, mod(f, nf) + 1), uu(1, 1, f), vv(1, 1, f))
  end do
  open (newunit=u, file=trim(dir) // '/dropin_out.bin', access='stream', form='unformatted', status='replace')
  write (u) gk1, gk2, sp, gy, sy, sx, v1, d1, v2, d2, uu, vv
  close (u)
  print '(a)', 'sml_dropin_check ok'
end program
