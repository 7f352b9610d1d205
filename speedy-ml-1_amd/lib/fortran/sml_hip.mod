﻿!mod$ v1 sum:09b20f0812bc218b
!need$ 0bde2ac47243ead2 i iso_c_binding
module sml_hip
use,intrinsic::iso_c_binding,only:c_associated
use,intrinsic::iso_c_binding,only:c_funloc
use,intrinsic::iso_c_binding,only:c_funptr
use,intrinsic::iso_c_binding,only:c_f_pointer
use,intrinsic::iso_c_binding,only:c_loc
use,intrinsic::iso_c_binding,only:c_null_funptr
use,intrinsic::iso_c_binding,only:c_null_ptr
use,intrinsic::iso_c_binding,only:c_ptr
use,intrinsic::iso_c_binding,only:c_sizeof
use,intrinsic::iso_c_binding,only:operator(==)
use,intrinsic::iso_c_binding,only:operator(/=)
use,intrinsic::iso_c_binding,only:c_int8_t
use,intrinsic::iso_c_binding,only:c_int16_t
use,intrinsic::iso_c_binding,only:c_int32_t
use,intrinsic::iso_c_binding,only:c_int64_t
use,intrinsic::iso_c_binding,only:c_int128_t
use,intrinsic::iso_c_binding,only:c_int
use,intrinsic::iso_c_binding,only:c_short
use,intrinsic::iso_c_binding,only:c_long
use,intrinsic::iso_c_binding,only:c_long_long
use,intrinsic::iso_c_binding,only:c_signed_char
use,intrinsic::iso_c_binding,only:c_size_t
use,intrinsic::iso_c_binding,only:c_intmax_t
use,intrinsic::iso_c_binding,only:c_intptr_t
use,intrinsic::iso_c_binding,only:c_ptrdiff_t
use,intrinsic::iso_c_binding,only:c_int_least8_t
use,intrinsic::iso_c_binding,only:c_int_fast8_t
use,intrinsic::iso_c_binding,only:c_int_least16_t
use,intrinsic::iso_c_binding,only:c_int_fast16_t
use,intrinsic::iso_c_binding,only:c_int_least32_t
use,intrinsic::iso_c_binding,only:c_int_fast32_t
use,intrinsic::iso_c_binding,only:c_int_least64_t
use,intrinsic::iso_c_binding,only:c_int_fast64_t
use,intrinsic::iso_c_binding,only:c_int_least128_t
use,intrinsic::iso_c_binding,only:c_int_fast128_t
use,intrinsic::iso_c_binding,only:c_float
use,intrinsic::iso_c_binding,only:c_double
use,intrinsic::iso_c_binding,only:c_long_double
use,intrinsic::iso_c_binding,only:c_float_complex
use,intrinsic::iso_c_binding,only:c_double_complex
use,intrinsic::iso_c_binding,only:c_long_double_complex
use,intrinsic::iso_c_binding,only:c_bool
use,intrinsic::iso_c_binding,only:c_char
use,intrinsic::iso_c_binding,only:c_null_char
use,intrinsic::iso_c_binding,only:c_alert
use,intrinsic::iso_c_binding,only:c_backspace
use,intrinsic::iso_c_binding,only:c_form_feed
use,intrinsic::iso_c_binding,only:c_new_line
use,intrinsic::iso_c_binding,only:c_carriage_return
use,intrinsic::iso_c_binding,only:c_horizontal_tab
use,intrinsic::iso_c_binding,only:c_vertical_tab
use,intrinsic::iso_c_binding,only:c_float128
use,intrinsic::iso_c_binding,only:c_float128_complex
use,intrinsic::iso_c_binding,only:c_uint8_t
use,intrinsic::iso_c_binding,only:c_uint16_t
use,intrinsic::iso_c_binding,only:c_uint32_t
use,intrinsic::iso_c_binding,only:c_uint64_t
use,intrinsic::iso_c_binding,only:c_uint128_t
use,intrinsic::iso_c_binding,only:c_unsigned_char
use,intrinsic::iso_c_binding,only:c_unsigned_short
use,intrinsic::iso_c_binding,only:c_unsigned
use,intrinsic::iso_c_binding,only:c_unsigned_long
use,intrinsic::iso_c_binding,only:c_unsigned_long_long
use,intrinsic::iso_c_binding,only:c_uintmax_t
use,intrinsic::iso_c_binding,only:c_uint_fast8_t
use,intrinsic::iso_c_binding,only:c_uint_fast16_t
use,intrinsic::iso_c_binding,only:c_uint_fast32_t
use,intrinsic::iso_c_binding,only:c_uint_fast64_t
use,intrinsic::iso_c_binding,only:c_uint_fast128_t
use,intrinsic::iso_c_binding,only:c_uint_least8_t
use,intrinsic::iso_c_binding,only:c_uint_least16_t
use,intrinsic::iso_c_binding,only:c_uint_least32_t
use,intrinsic::iso_c_binding,only:c_uint_least64_t
use,intrinsic::iso_c_binding,only:c_uint_least128_t
use,intrinsic::iso_c_binding,only:c_f_procpointer
integer(4),parameter::sml_ok=0_4
integer(4),parameter::sml_f32=1_4
integer(4),parameter::sml_f64=2_4
integer(4),parameter::sml_spec_field=1984_4
integer(4),parameter::sml_grid_field=4608_4
interface
function sml_last_error() bind(c,name="sml_last_error") result(p)
import::c_ptr
type(c_ptr)::p
end
end interface
interface
function sml_abi_version() bind(c,name="sml_abi_version") result(v)
integer(4)::v
end
end interface
interface
function sml_spectral_create(radius,ctx) bind(c,name="sml_spectral_create") result(rc)
import::c_ptr
real(8),value::radius
type(c_ptr)::ctx
integer(4)::rc
end
end interface
interface
function sml_spectral_destroy(ctx) bind(c,name="sml_spectral_destroy") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(4)::rc
end
end interface
interface
function sml_grid_host(ctx,spec,grid,nf,kcos) bind(c,name="sml_grid_host") result(rc)
import::c_ptr
type(c_ptr),value::ctx
real(8),intent(in)::spec(1_8:*)
real(8),intent(out)::grid(1_8:*)
integer(4),value::nf
integer(4),value::kcos
integer(4)::rc
end
end interface
interface
function sml_spec_host(ctx,grid,spec,nf) bind(c,name="sml_spec_host") result(rc)
import::c_ptr
type(c_ptr),value::ctx
real(8),intent(in)::grid(1_8:*)
real(8),intent(out)::spec(1_8:*)
integer(4),value::nf
integer(4)::rc
end
end interface
interface
function sml_grid_batched(ctx,d_spec,d_grid,nf,kcos,stream) bind(c,name="sml_grid_batched") result(rc)
import::c_ptr
type(c_ptr),value::ctx
type(c_ptr),value::d_spec
type(c_ptr),value::d_grid
integer(4),value::nf
integer(4),value::kcos
type(c_ptr),value::stream
integer(4)::rc
end
end interface
interface
function sml_spec_batched(ctx,d_grid,d_spec,nf,stream) bind(c,name="sml_spec_batched") result(rc)
import::c_ptr
type(c_ptr),value::ctx
type(c_ptr),value::d_grid
type(c_ptr),value::d_spec
integer(4),value::nf
type(c_ptr),value::stream
integer(4)::rc
end
end interface
interface
function sml_res_create(numregions,nlocal,region_ids,sst_flags,n,k,chunk_speedy,nout,weight_dtype,leakage,ctx) bind(c,name="sml_res_create") result(rc)
import::c_ptr
integer(4),value::numregions
integer(4),value::nlocal
integer(4),intent(in)::region_ids(1_8:*)
integer(1),intent(in)::sst_flags(1_8:*)
integer(4),intent(in)::n(1_8:*)
integer(4),intent(in)::k(1_8:*)
integer(4),value::chunk_speedy
integer(4),value::nout
integer(4),value::weight_dtype
real(8),value::leakage
type(c_ptr)::ctx
integer(4)::rc
end
end interface
interface
function sml_res_destroy(ctx) bind(c,name="sml_res_destroy") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(4)::rc
end
end interface
interface
function sml_res_ninp(ctx,i,ninp) bind(c,name="sml_res_ninp") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(4),value::i
integer(4),intent(out)::ninp
integer(4)::rc
end
end interface
interface
function sml_res_feedback_offsets(ctx,offsets) bind(c,name="sml_res_feedback_offsets") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(8),intent(out)::offsets(1_8:*)
integer(4)::rc
end
end interface
interface
function sml_res_load_region_f32(ctx,i,rows,cols,vals,win,wout,mean,std) bind(c,name="sml_res_load_region_f32") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(4),value::i
integer(4),intent(in)::rows(1_8:*)
integer(4),intent(in)::cols(1_8:*)
real(4),intent(in)::vals(1_8:*)
real(4),intent(in)::win(1_8:*)
real(4),intent(in)::wout(1_8:*)
real(8),intent(in)::mean(1_8:*)
real(8),intent(in)::std(1_8:*)
integer(4)::rc
end
end interface
interface
function sml_res_load_region_f64(ctx,i,rows,cols,vals,win,wout,mean,std) bind(c,name="sml_res_load_region_f64") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(4),value::i
integer(4),intent(in)::rows(1_8:*)
integer(4),intent(in)::cols(1_8:*)
real(8),intent(in)::vals(1_8:*)
real(8),intent(in)::win(1_8:*)
real(8),intent(in)::wout(1_8:*)
real(8),intent(in)::mean(1_8:*)
real(8),intent(in)::std(1_8:*)
integer(4)::rc
end
end interface
interface
function sml_res_set_state(ctx,i,x) bind(c,name="sml_res_set_state") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(4),value::i
real(8),intent(in)::x(1_8:*)
integer(4)::rc
end
end interface
interface
function sml_res_get_state(ctx,i,x) bind(c,name="sml_res_get_state") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(4),value::i
real(8),intent(out)::x(1_8:*)
integer(4)::rc
end
end interface
interface
function sml_res_step_host(ctx,feedback,local_model,outvec) bind(c,name="sml_res_step_host") result(rc)
import::c_ptr
type(c_ptr),value::ctx
real(8),intent(in)::feedback(1_8:*)
real(8),intent(in)::local_model(1_8:*)
real(8),intent(out)::outvec(1_8:*)
integer(4)::rc
end
end interface
interface
function sml_res_step(ctx,d_feedback,d_local_model,d_outvec,stream) bind(c,name="sml_res_step") result(rc)
import::c_ptr
type(c_ptr),value::ctx
type(c_ptr),value::d_feedback
type(c_ptr),value::d_local_model
type(c_ptr),value::d_outvec
type(c_ptr),value::stream
integer(4)::rc
end
end interface
interface
function sml_res_step_begin(ctx,d_feedback,stream) bind(c,name="sml_res_step_begin") result(rc)
import::c_ptr
type(c_ptr),value::ctx
type(c_ptr),value::d_feedback
type(c_ptr),value::stream
integer(4)::rc
end
end interface
interface
function sml_res_step_finish_grid(ctx,d_fc4d,d_fc2d,d_local_model,d_outvec,stream) bind(c,name="sml_res_step_finish_grid") result(rc)
import::c_ptr
type(c_ptr),value::ctx
type(c_ptr),value::d_fc4d
type(c_ptr),value::d_fc2d
type(c_ptr),value::d_local_model
type(c_ptr),value::d_outvec
type(c_ptr),value::stream
integer(4)::rc
end
end interface
interface
function sml_res_set_read_waves(ctx,waves) bind(c,name="sml_res_set_read_waves") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(4),value::waves
integer(4)::rc
end
end interface
interface
function sml_stream_create_cu_range(first_cu,num_cus,stream) bind(c,name="sml_stream_create_cu_range") result(rc)
import::c_ptr
integer(4),value::first_cu
integer(4),value::num_cus
type(c_ptr)::stream
integer(4)::rc
end
end interface
interface
function sml_stream_destroy(stream) bind(c,name="sml_stream_destroy") result(rc)
import::c_ptr
type(c_ptr),value::stream
integer(4)::rc
end
end interface
interface
function sml_res_step_finish(ctx,d_local_model,d_outvec,stream) bind(c,name="sml_res_step_finish") result(rc)
import::c_ptr
type(c_ptr),value::ctx
type(c_ptr),value::d_local_model
type(c_ptr),value::d_outvec
type(c_ptr),value::stream
integer(4)::rc
end
end interface
interface
function sml_nc_read_region(path,dims,win,wout,rows,cols,vals,mean,std) bind(c,name="sml_nc_read_region") result(rc)
import::c_ptr
character(1_8,1),intent(in)::path(1_8:*)
integer(8),intent(out)::dims(1_8:6_8)
type(c_ptr),value::win
type(c_ptr),value::wout
type(c_ptr),value::rows
type(c_ptr),value::cols
type(c_ptr),value::vals
type(c_ptr),value::mean
type(c_ptr),value::std
integer(4)::rc
end
end interface
interface
function sml_dyn_create(radius,ctx) bind(c,name="sml_dyn_create") result(rc)
import::c_ptr
real(8),value::radius
type(c_ptr),intent(out)::ctx
integer(4)::rc
end
end interface
interface
function sml_dyn_destroy(ctx) bind(c,name="sml_dyn_destroy") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(4)::rc
end
end interface
interface
function sml_dyn_impint(ctx,dt,alph) bind(c,name="sml_dyn_impint") result(rc)
import::c_ptr
type(c_ptr),value::ctx
real(8),value::dt
real(8),value::alph
integer(4)::rc
end
end interface
interface
function sml_dyn_set_forcing(ctx,phis,tcorh,qcorh) bind(c,name="sml_dyn_set_forcing") result(rc)
import::c_ptr
type(c_ptr),value::ctx
complex(8),intent(in)::phis(1_8:*)
complex(8),intent(in)::tcorh(1_8:*)
complex(8),intent(in)::qcorh(1_8:*)
integer(4)::rc
end
end interface
interface
function sml_dyn_set_state(ctx,vor,div,t,ps,tr) bind(c,name="sml_dyn_set_state") result(rc)
import::c_ptr
type(c_ptr),value::ctx
complex(8),intent(in)::vor(1_8:*)
complex(8),intent(in)::div(1_8:*)
complex(8),intent(in)::t(1_8:*)
complex(8),intent(in)::ps(1_8:*)
complex(8),intent(in)::tr(1_8:*)
integer(4)::rc
end
end interface
interface
function sml_dyn_get_state(ctx,vor,div,t,ps,tr) bind(c,name="sml_dyn_get_state") result(rc)
import::c_ptr
type(c_ptr),value::ctx
complex(8),intent(out)::vor(1_8:*)
complex(8),intent(out)::div(1_8:*)
complex(8),intent(out)::t(1_8:*)
complex(8),intent(out)::ps(1_8:*)
complex(8),intent(out)::tr(1_8:*)
integer(4)::rc
end
end interface
interface
function sml_dyn_window(ctx,nleap,delt,alph,rob,wil,stream) bind(c,name="sml_dyn_window") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(4),value::nleap
real(8),value::delt
real(8),value::alph
real(8),value::rob
real(8),value::wil
type(c_ptr),value::stream
integer(4)::rc
end
end interface
interface
function sml_dyn_step_host(ctx,j1,j2,dt,alph,rob,wil,phys) bind(c,name="sml_dyn_step_host") result(rc)
import::c_ptr
type(c_ptr),value::ctx
integer(4),value::j1
integer(4),value::j2
real(8),value::dt
real(8),value::alph
real(8),value::rob
real(8),value::wil
real(8),intent(in)::phys(1_8:*)
integer(4)::rc
end
end interface
interface
function sml_dyn_from_grid_host(ctx,grid4d,logp,minmax,safe) bind(c,name="sml_dyn_from_grid_host") result(rc)
import::c_ptr
type(c_ptr),value::ctx
real(8),intent(in)::grid4d(1_8:*)
real(8),intent(in)::logp(1_8:*)
real(8),intent(out)::minmax(1_8:8_8)
integer(4),intent(out)::safe
integer(4)::rc
end
end interface
interface
function sml_dyn_to_grid_host(ctx,grid4d,logp) bind(c,name="sml_dyn_to_grid_host") result(rc)
import::c_ptr
type(c_ptr),value::ctx
real(8),intent(out)::grid4d(1_8:*)
real(8),intent(out)::logp(1_8:*)
integer(4)::rc
end
end interface
contains
subroutine sml_check(rc,what)
integer(4),intent(in)::rc
character(*,1),intent(in)::what
end
subroutine sml_read_trained_res(ctx,i,filename)
type(c_ptr),intent(in)::ctx
integer(4),intent(in)::i
character(*,1),intent(in)::filename
end
subroutine sml_predict_all(ctx,feedback,local_model,outvec)
type(c_ptr),intent(in)::ctx
real(8),intent(in)::feedback(:)
real(8),intent(in)::local_model(:,:)
real(8),intent(out)::outvec(:,:)
end
end
