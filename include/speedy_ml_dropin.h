/*
 * speedy_ml_dropin.h -- libspeedyml_dropin.so: the reference's single-field spectral
 * subroutines under their Fortran (flang / gfortran) symbols, for a host that links
 * the reference's own callers against the GPU path instead of spe_spectral.o /
 * spe_subfft_fftpack.o.  Arguments by reference, Fortran column-major arrays, no
 * status (an error prints the library's message and exits, as the reference's own
 * failures stop).  One field per call, synchronous (H2D, GPU kernels, D2H).
 *
 *   grid_    <- grid(vorm, vorg, kcos)          src/spe_spectral.f90:389-401
 *   spec_    <- spec(vorg, vorm)                src/spe_spectral.f90:403-414
 *   vdspec_  <- vdspec(ug, vg, vorm, divm, kcos) src/spe_spectral.f90:416-452
 *   uvspec_  <- uvspec(vorm, divm, ucosm, vcosm) src/spe_spectral.f90:351-387
 *   gridy_   <- gridy(v, varm)                  src/spe_spectral.f90:454-495
 *   specy_   <- specy(varm, vorm)               src/spe_spectral.f90:497-538
 *   gridx_   <- gridx(varm, vorg, kcos)         src/spe_subfft_fftpack.f90:15-51
 *   specx_   <- specx(vorg, varm)               src/spe_subfft_fftpack.f90:55-87
 *
 * vorm/divm/ucosm/vcosm: real(mx2=62, nx=32); vorg/ug/vg: real(ix=96, il=48);
 * varm: real(mx2=62, il=48).  The tables are those of parmtr(rearth) + inifft,
 * built on first use; sml_dropin_init(radius) rebuilds them for another radius
 * (the explicit init the module-global tables of mod_spectral need).
 */
#ifndef SPEEDY_ML_DROPIN_H
#define SPEEDY_ML_DROPIN_H

#ifdef __cplusplus
extern "C" {
#endif

int sml_dropin_init(double radius);
void grid_(const double *vorm, double *vorg, const int *kcos);
void spec_(const double *vorg, double *vorm);
void vdspec_(const double *ug, const double *vg, double *vorm, double *divm, const int *kcos);
void uvspec_(const double *vorm, const double *divm, double *ucosm, double *vcosm);
void gridy_(const double *v, double *varm);
void specy_(const double *varm, double *vorm);
void gridx_(const double *varm, double *vorg, const int *kcos);
void specx_(const double *vorg, double *varm);

#ifdef __cplusplus
}
#endif
#endif /* SPEEDY_ML_DROPIN_H */
