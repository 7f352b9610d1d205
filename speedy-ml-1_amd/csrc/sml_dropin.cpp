// sml_dropin.cpp -- libspeedyml_dropin.so: the reference's single-field spectral
// subroutines under their own Fortran symbols, so a host built from the reference's
// sources links this library in place of spe_spectral.o / spe_subfft_fftpack.o.
//
// Reference seam: grid, spec, vdspec, uvspec, gridy, specy
// (src/spe_spectral.f90:351-538) and gridx, specx (src/spe_subfft_fftpack.f90:15-87)
// are external implicit-interface subroutines: arguments by reference, column-major
// arrays, no status return, one field per call, tables in module globals.  Here each
// call is one batched launch of nfields = 1 on the GPU (H2D, kernels, D2H), through a
// process-wide spectral context built on first use with the Earth radius of
// mod_dyncon1 (rearth = 6.371e6) or by sml_dropin_init(radius) -- the explicit init
// after parmtr that the module-global tables require.  Errors stop the program with
// the library's message, as the reference's own failures do (print + stop).
//
// The single-field calls are for parity and for hosts that keep the reference's
// call structure; the hot path batches (include/speedy_ml.h).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <mutex>

#include "../../include/speedy_ml.h"
#include "../../include/speedy_ml_dropin.h"

namespace {

constexpr int kSF = SML_SPEC_FIELD, kGF = SML_GRID_FIELD, kVF = SML_MX2 * SML_IL;

struct DropIn {
    sml_spectral *sp = nullptr;
    double *d = nullptr;  // [2 grid | 2 spec | 2 varm] scratch
    double radius = 6.371e6;
};
DropIn g_drop;
std::mutex g_mu;

[[noreturn]] void die(const char *what) {
    std::fprintf(stderr, "speedyml drop-in %s failed: %s\n", what, sml_last_error());
    std::exit(1);
}

void ok(int rc, const char *what) {
    if (rc != SML_OK) die(what);
}

void hip_ok(hipError_t e, const char *what) {
    if (e != hipSuccess) {
        std::fprintf(stderr, "speedyml drop-in %s failed: %s\n", what, hipGetErrorString(e));
        std::exit(1);
    }
}

DropIn &ctx() {
    if (!g_drop.sp) {
        ok(sml_spectral_create(g_drop.radius, &g_drop.sp), "sml_spectral_create");
        // the scratch does not depend on the radius: allocated once, kept over re-inits
        if (!g_drop.d) hip_ok(hipMalloc(&g_drop.d, sizeof(double) * (2 * kGF + 2 * kSF + 2 * kVF)), "hipMalloc");
    }
    return g_drop;
}

double *dgrid(int i) { return g_drop.d + (size_t)i * kGF; }
double *dspec(int i) { return g_drop.d + 2 * (size_t)kGF + (size_t)i * kSF; }
double *dvarm(int i) { return g_drop.d + 2 * (size_t)kGF + 2 * (size_t)kSF + (size_t)i * kVF; }

void h2d(double *d, const double *h, int n) { hip_ok(hipMemcpy(d, h, sizeof(double) * n, hipMemcpyHostToDevice), "H2D"); }
void d2h(double *h, const double *d, int n) { hip_ok(hipMemcpy(h, d, sizeof(double) * n, hipMemcpyDeviceToHost), "D2H"); }

}  // namespace

extern "C" int sml_dropin_init(double radius) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_drop.sp) {
        sml_spectral_destroy(g_drop.sp);
        g_drop.sp = nullptr;
    }
    g_drop.radius = radius;
    ctx();
    return SML_OK;
}

// grid(vorm, vorg, kcos): spe_spectral.f90:389-401
extern "C" void grid_(const double *vorm, double *vorg, const int *kcos) {
    std::lock_guard<std::mutex> lk(g_mu);
    DropIn &c = ctx();
    h2d(dspec(0), vorm, kSF);
    ok(sml_grid_batched(c.sp, dspec(0), dgrid(0), 1, *kcos, nullptr), "grid");
    d2h(vorg, dgrid(0), kGF);
}

// spec(vorg, vorm): :403-414
extern "C" void spec_(const double *vorg, double *vorm) {
    std::lock_guard<std::mutex> lk(g_mu);
    DropIn &c = ctx();
    h2d(dgrid(0), vorg, kGF);
    ok(sml_spec_batched(c.sp, dgrid(0), dspec(0), 1, nullptr), "spec");
    d2h(vorm, dspec(0), kSF);
}

// vdspec(ug, vg, vorm, divm, kcos): :416-452
extern "C" void vdspec_(const double *ug, const double *vg, double *vorm, double *divm, const int *kcos) {
    std::lock_guard<std::mutex> lk(g_mu);
    DropIn &c = ctx();
    h2d(dgrid(0), ug, kGF);
    h2d(dgrid(1), vg, kGF);
    ok(sml_vdspec_batched(c.sp, dgrid(0), dgrid(1), dspec(0), dspec(1), 1, *kcos, nullptr), "vdspec");
    d2h(vorm, dspec(0), kSF);
    d2h(divm, dspec(1), kSF);
}

// uvspec(vorm, divm, ucosm, vcosm): :351-387
extern "C" void uvspec_(const double *vorm, const double *divm, double *ucosm, double *vcosm) {
    std::lock_guard<std::mutex> lk(g_mu);
    DropIn &c = ctx();
    h2d(dspec(0), vorm, kSF);
    h2d(dspec(1), divm, kSF);
    ok(sml_uvspec_batched(c.sp, dspec(0), dspec(1), dgrid(0), dgrid(1), 1, nullptr), "uvspec");
    d2h(ucosm, dgrid(0), kSF);
    d2h(vcosm, dgrid(1), kSF);
}

// gridy(v, varm): :454-495
extern "C" void gridy_(const double *v, double *varm) {
    std::lock_guard<std::mutex> lk(g_mu);
    DropIn &c = ctx();
    h2d(dspec(0), v, kSF);
    ok(sml_gridy_batched(c.sp, dspec(0), dvarm(0), 1, nullptr), "gridy");
    d2h(varm, dvarm(0), kVF);
}

// specy(varm, vorm): :497-538
extern "C" void specy_(const double *varm, double *vorm) {
    std::lock_guard<std::mutex> lk(g_mu);
    DropIn &c = ctx();
    h2d(dvarm(0), varm, kVF);
    ok(sml_specy_batched(c.sp, dvarm(0), dspec(0), 1, nullptr), "specy");
    d2h(vorm, dspec(0), kSF);
}

// gridx(varm, vorg, kcos): spe_subfft_fftpack.f90:15-51
extern "C" void gridx_(const double *varm, double *vorg, const int *kcos) {
    std::lock_guard<std::mutex> lk(g_mu);
    DropIn &c = ctx();
    h2d(dvarm(0), varm, kVF);
    ok(sml_gridx_batched(c.sp, dvarm(0), dgrid(0), 1, *kcos, nullptr), "gridx");
    d2h(vorg, dgrid(0), kGF);
}

// specx(vorg, varm): spe_subfft_fftpack.f90:55-87
extern "C" void specx_(const double *vorg, double *varm) {
    std::lock_guard<std::mutex> lk(g_mu);
    DropIn &c = ctx();
    h2d(dgrid(0), vorg, kGF);
    ok(sml_specx_batched(c.sp, dgrid(0), dvarm(0), 1, nullptr), "specx");
    d2h(varm, dvarm(0), kVF);
}
