"""speedy_res_interface with the reference's own types: the reference's callers
compile against the build's Fortran modules unchanged (CPU; AMD flang).

* /root/reference/src/dyn_stloop.f90 -- `use speedy_res_interface, only :
  getspeedyvariable` -- compiled AS-IS against the build's speedy_res_interface,
  with the reference's own SPEEDY modules it uses (mod_atparam, mod_lflags,
  mod_tsteps, mod_date, mod_dynvar) compiled as-is beside it; only
  `mod_reservoir, only : global_time_step` (a CPU reservoir module the GPU path
  replaces) is a one-variable module written here.
* a caller written like parallelmain.f90:9-11 (`use speedy_res_interface, only :
  startspeedy`, `use mod_utilities, only : main_type, dp`, `type(main_type) :: res`,
  `call startspeedy(res%model_parameters, res%grid(i,j), runspeedy)`), and a module
  procedure written like mod_reservoir.f90:334/360/566/614/653 (`reservoir`,
  `model_parameters`, `grid` of mod_utilities' types; read_era /
  read_model_states / read_era_netcdf_opened with the reference's argument lists,
  `calendar` from mod_calendar): compiled and linked.
* the linked parallelmain-style caller runs on the CPU: startspeedy's
  initializedomain(mpi_res%numprocs, mpi_res%proc_num, ...) (speedy_res_interface.f90:36)
  gives, with a 1152-rank world, region proc_num's extents
  (speedy_ml_amd.domain.region_geometry), and mod_calendar's
  get_current_time_delta_hour matches the library's calendar.

Skipped when /root/reference is absent (the GPU box)."""
import os
import subprocess

import numpy as np
import pytest

from speedy_ml_amd import _lib, domain

REF = "/root/reference/src"
FLANG = "/opt/rocm/lib/llvm/bin/flang"
FDIR = os.path.join(_lib.PKG_ROOT, "fortran")
MODDIR = os.path.join(_lib.PKG_ROOT, "lib", "fortran")
IFACE_OBJS = ["speedy_res_interface.o", "mod_utilities.o", "mod_calendar.o", "mpires.o", "resdomain.o", "sml_hip.o"]

pytestmark = pytest.mark.skipif(not os.path.isdir(REF) or not os.path.exists(FLANG),
                                reason="needs the reference sources and AMD flang")

PARALLELMAIN_LIKE = """
program parallelmain_like
  ! the use lines of parallelmain.f90:9-11 that touch the interface and its types
  use speedy_res_interface, only : startspeedy
  use mod_utilities, only : main_type, dp
  use mod_calendar
  use mpires, only : set_world
  implicit none
  type(main_type) :: res
  logical :: runspeedy = .False.
  integer :: i, j, r, u, regs(6)
  real(kind=dp) :: x
  regs = [0, 23, 24, 500, 954, 1151]
  res%model_parameters%number_of_regions = 1152
  res%model_parameters%overlap = 1
  allocate(res%grid(1, 1), res%reservoir(1, 1))
  i = 1
  j = 1
  res%grid(i, j)%num_vert_levels = 1
  res%grid(i, j)%vert_overlap = 0
  open(newunit=u, file='extents.txt', status='replace')
  do r = 1, size(regs)
    call set_world(1152, regs(r))
    call startspeedy(res%model_parameters, res%grid(i, j), runspeedy)
    write(u, '(21i6)') regs(r), res%grid(i,j)%res_xstart, res%grid(i,j)%res_xend, res%grid(i,j)%res_ystart, &
      res%grid(i,j)%res_yend, res%grid(i,j)%resxchunk, res%grid(i,j)%resychunk, res%grid(i,j)%input_xstart, &
      res%grid(i,j)%input_xend, res%grid(i,j)%input_ystart, res%grid(i,j)%input_yend, res%grid(i,j)%inputxchunk, &
      res%grid(i,j)%inputychunk, res%grid(i,j)%tdata_xstart, res%grid(i,j)%tdata_xend, res%grid(i,j)%tdata_ystart, &
      res%grid(i,j)%tdata_yend, res%grid(i,j)%res_zstart, res%grid(i,j)%res_zend, res%grid(i,j)%inputzchunk, &
      merge(1, 0, res%grid(i,j)%bottom)
  end do
  close(u)
  open(newunit=u, file='calendar.txt', status='replace')
  do r = 0, 40
    call get_current_time_delta_hour(calendar, 86184 + 997 * r)
    write(u, '(5i8)') 86184 + 997 * r, calendar%currentyear, calendar%currentmonth, calendar%currentday, &
      calendar%currenthour
  end do
  close(u)
  x = 0.0_dp
  print *, 'parallelmain_like ok', x
end program
"""

MOD_RESERVOIR_LIKE = """
module mod_reservoir_like
  use mod_utilities, only : dp, reservoir_type, model_parameters_type, grid_type, era_data_type, &
                            speedy_data_type, opened_netcdf_type
  use mod_calendar
  implicit none
contains
  subroutine get_training_data(reservoir, model_parameters, grid, start_year)
    ! the interface calls of mod_reservoir.f90:334-360, 566 and 614-653, 761
    use speedy_res_interface, only : read_era, read_model_states, read_era_netcdf_opened
    type(reservoir_type), intent(inout)        :: reservoir
    type(model_parameters_type), intent(inout) :: model_parameters
    type(grid_type), intent(inout)             :: grid
    integer, intent(in)                        :: start_year
    type(era_data_type)    :: era_data
    type(speedy_data_type) :: speedy_data
    type(opened_netcdf_type), allocatable :: netcdf_files(:)
    call initialize_calendar(calendar,1981,1,1,0)
    call get_current_time_delta_hour(calendar,model_parameters%discardlength+model_parameters%traininglength+model_parameters%synclength)
    call read_era(reservoir,grid,model_parameters,calendar%startyear,calendar%currentyear,era_data)
    call read_model_states(reservoir,grid,model_parameters,calendar%startyear,calendar%currentyear,speedy_data)
    call read_era(reservoir,grid,model_parameters,start_year,calendar%currentyear,era_data,1)
    call read_model_states(reservoir,grid,model_parameters,start_year,calendar%currentyear,speedy_data,1)
    allocate(netcdf_files(1))
    call read_era_netcdf_opened(reservoir,grid,model_parameters,start_year,calendar%currentyear,era_data, &
                                netcdf_files,1)
    reservoir%feedback = era_data%era_logp(1, 1, :)
  end subroutine
end module
"""

GLOBAL_TIME_STEP = """
module mod_reservoir
  ! the one variable dyn_stloop.f90:15 takes from the reference's CPU reservoir module
  integer :: global_time_step = 6
end module
"""


def _run(cmd, cwd):
    p = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    assert p.returncode == 0, f"{' '.join(cmd)}\n{p.stdout[-3000:]}\n{p.stderr[-3000:]}"
    return p


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    _run(["make", "-s", "-C", FDIR], FDIR)
    return MODDIR


def test_reference_dyn_stloop_compiles_unchanged(built, tmp_path):
    mods = ["mod_atparam", "mod_lflags", "mod_tsteps", "mod_date", "mod_dynvar"]
    _run([FLANG, "-c", "-fdefault-real-8", "-w"] + [os.path.join(REF, m + ".f90") for m in mods], str(tmp_path))
    (tmp_path / "mod_reservoir_gts.f90").write_text(GLOBAL_TIME_STEP)
    _run([FLANG, "-c", "mod_reservoir_gts.f90"], str(tmp_path))
    _run([FLANG, "-c", "-fdefault-real-8", "-w", f"-I{built}", "-I.", os.path.join(REF, "dyn_stloop.f90"),
          "-o", "dyn_stloop.o"], str(tmp_path))
    assert (tmp_path / "dyn_stloop.o").exists()


def test_reference_style_callers_compile_link_and_run(built, tmp_path):
    (tmp_path / "caller_main.f90").write_text(PARALLELMAIN_LIKE)
    (tmp_path / "caller_res.f90").write_text(MOD_RESERVOIR_LIKE)
    objs = [os.path.join(built, o) for o in IFACE_OBJS]
    _run([FLANG, "-c", f"-I{built}", "caller_res.f90"], str(tmp_path))
    lib = os.path.dirname(_lib.LIB_PATH)
    _run([FLANG, f"-I{built}", "-I.", "caller_main.f90", "caller_res.o"] + objs
         + [f"-L{lib}", "-lspeedyml", f"-Wl,-rpath,{lib}", "-o", "caller"], str(tmp_path))
    p = _run([str(tmp_path / "caller")], str(tmp_path))
    assert "parallelmain_like ok" in p.stdout
    ext = np.loadtxt(tmp_path / "extents.txt", dtype=int)
    for row in ext:
        g = domain.region_geometry(int(row[0]))
        assert list(row[1:13]) == [g.res_xstart, g.res_xend, g.res_ystart, g.res_yend, g.resx, g.resy,
                                   g.in_xstart, g.in_xend, g.in_ystart, g.in_yend, g.inx, g.iny], row
        # tdata: the resolved 2x2 inside the input tile (get_trainingdataindices)
        tx0, tx1, ty0, ty1 = row[13:17]
        assert (tx0, tx1) == (2, g.inx - 1)
        assert ty1 - ty0 + 1 == g.resy and ty0 == (g.res_ystart - g.in_ystart + 1)
        assert list(row[17:21]) == [1, 8, 8, 1]  # one vertical level: z 1..8, bottom
    import ctypes

    cal = np.loadtxt(tmp_path / "calendar.txt", dtype=int)
    feb = ctypes.c_int(0)
    for h, y, m, d, hr in cal:
        date = (ctypes.c_int * 4)()
        assert _lib.lib().sml_calendar_delta_hour(1981, int(h), ctypes.byref(feb), date) == 0
        assert list(date) == [y, m, d, hr], (h, list(date), (y, m, d, hr))
