!> mod_calendar -- the hybrid's own calendar (src/mod_calendar.f90:1-22, 24-92),
!> independent of SPEEDY's: the module's `calendar`, initialize_calendar (start date
!> only, as the reference: the current date is left as it was) and
!> get_current_time_delta_hour.  The arithmetic is the library's
!> sml_calendar_delta_hour (csrc/sml_hybrid.hip, with the reference's quirks: years of
!> 8760 h, the elapsed leap days subtracted, an exact month boundary falling to the
!> last day of the month before); the reference's SAVEd month table -- February
!> latched at 29 days once a leap year is met -- is this module's `feb29_latch`,
!> shared by every call of the process as there.
module mod_calendar
  use iso_c_binding
  use mod_utilities, only: calendar_type
  use sml_hip, only: sml_check
  implicit none

  type(calendar_type) :: calendar
  integer(c_int) :: feb29_latch = 0

  interface
    function sml_calendar_delta_hour(startyear, hours_elapsed, feb29, date) bind(C, name='sml_calendar_delta_hour') &
        result(rc)
      import :: c_int, c_int64_t
      integer(c_int), value :: startyear
      integer(c_int64_t), value :: hours_elapsed
      integer(c_int), intent(inout) :: feb29
      integer(c_int), intent(out) :: date(4)
      integer(c_int) :: rc
    end function
  end interface

contains

  subroutine initialize_calendar(datetime, startyear, startmonth, startday, starthour)
    type(calendar_type), intent(inout) :: datetime
    integer, intent(in) :: startyear, startmonth, startday, starthour
    datetime%startyear = startyear
    datetime%startmonth = startmonth
    datetime%startday = startday
    datetime%starthour = starthour
  end subroutine

  subroutine get_current_time_delta_hour(datetime, hours_elapsed)
    type(calendar_type), intent(inout) :: datetime
    integer, intent(in) :: hours_elapsed
    integer(c_int) :: d(4)
    call sml_check(sml_calendar_delta_hour(int(datetime%startyear, c_int), int(hours_elapsed, c_int64_t), &
                                           feb29_latch, d), 'sml_calendar_delta_hour')
    datetime%currentyear = d(1)
    datetime%currentmonth = d(2)
    datetime%currentday = d(3)
    datetime%currenthour = d(4)
  end subroutine

  !> leap_year_check (:94-106)
  subroutine leap_year_check(year, is_leap_year)
    integer, intent(in) :: year
    logical, intent(out) :: is_leap_year
    is_leap_year = (mod(year, 4) == 0 .and. mod(year, 100) /= 0) .or. mod(year, 400) == 0
  end subroutine
end module mod_calendar
