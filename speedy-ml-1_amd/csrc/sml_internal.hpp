// sml_internal.hpp -- shared internals of libspeedyml (error state, HIP checks,
// region geometry).  Host-only; included by the .hip and .cpp translation units.
#pragma once

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/speedy_ml.h"

namespace sml {

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
void clear_error();
}  // namespace sml
struct sml_reservoirs;
namespace sml {
// the context holds every region, in global order (its local index is the region id)
bool res_in_global_order(const sml_reservoirs *c);
// sml_dynamics: the run_model exit's safety-check hand-off timed out (SML_ERR_STATE)
int dyn_check_late(sml_dynamics *d);
// the next sml_res_step_finish_grid / _finish_assemble launch waits in-kernel until
// *flag >= value (device words; *late set if it gave up), its weights loaded first
// (*late: a host-visible word; timeout in wall_clock64 ticks, 100 MHz)
int res_finish_wait(sml_reservoirs *c, const uint64_t *flag, uint64_t value, unsigned *late, long long timeout);
// the next sml_dyn_run_model / sml_dyn_from_grid waits in-kernel (its entry specx)
// until *flag >= value before it reads its input grids
int dyn_run_model_wait(sml_dynamics *d, const uint64_t *flag, uint64_t value, unsigned *late, long long timeout);
// the give-up time of the run_model exit's wait for its safety check (ticks)
int dyn_set_check_timeout(sml_dynamics *d, long long timeout);
// the next run_model's exit is followed by a one-lane store of value to *flag (inside the
// window graph when the exit is captured there)
int dyn_run_model_exit_store(sml_dynamics *d, uint64_t *flag, uint64_t value);
int dyn_run_model_entry_signal(sml_dynamics *d, uint64_t *counter, int *adds);
int dyn_check_event(sml_dynamics *d, void **ev);  // a hipEvent_t

// --------------------------------------------------------------- geometry
// Restatement of the res_domain.f90 decomposition used by every reservoir of the
// bottom level (num_vert_levels = 1, overlap = 1):
//   domaindecomposition        res_domain.f90:258-280
//   getworkerlower_leftcorner  res_domain.f90:282-292
//   getxyresextent             res_domain.f90:123-141
//   getoverlapindices          res_domain.f90:155-204
// Indices are 1-based like the reference.
constexpr int kXGrid = 96, kYGrid = 48, kZGrid = 8, kVars = 4;
constexpr int kGrid4d = kVars * kXGrid * kYGrid * kZGrid;  // 147456
constexpr int kGrid2d = kXGrid * kYGrid;                   // 4608

struct RegionGeom {
    int res_xstart, res_xend, res_ystart, res_yend, resx, resy;
    int in_xstart, in_xend, in_ystart, in_yend, inx, iny;
    bool pole, periodic;
};

inline bool decompose(int numregions, int *fx, int *fy) {
    if (numregions <= 0 || (kXGrid * kYGrid) % numregions != 0) return false;
    int n = (kXGrid * kYGrid) / numregions;
    int fmax = 0;
    while ((fmax + 1) * (fmax + 1) <= n) ++fmax;
    for (int i = fmax; i >= 1; --i) {
        if (kYGrid % i) continue;
        *fy = i;
        if (n % i) continue;
        *fx = n / i;
        if (kXGrid % *fx == 0) return true;
    }
    return false;
}

inline bool region_geom(int numregions, int region, RegionGeom *g, int overlap = 1) {
    int fx, fy;
    if (!decompose(numregions, &fx, &fy) || region < 0 || region >= numregions) return false;
    const int ncol = kYGrid / fy;
    const int col = region % ncol, row = region / ncol;
    g->resx = fx;
    g->resy = fy;
    g->res_xstart = row * fx + 1;
    g->res_xend = (row + 1) * fx;
    g->res_ystart = col * fy + 1;
    g->res_yend = (col + 1) * fy;
    g->inx = fx + 2 * overlap;
    g->iny = fy + 2 * overlap;
    g->periodic = g->pole = false;
    if (g->res_xstart - overlap < 1) {
        g->in_xstart = kXGrid - overlap + 1;
        g->periodic = true;
    } else {
        g->in_xstart = g->res_xstart - overlap;
    }
    if (g->res_xend + overlap > kXGrid) {
        g->in_xend = overlap;
        g->periodic = true;
    } else {
        g->in_xend = g->res_xend + overlap;
    }
    if (g->res_ystart - overlap < 1) {
        g->in_ystart = 1;
        g->iny = fy + overlap + (g->res_ystart - 1);
        g->pole = true;
    } else {
        g->in_ystart = g->res_ystart - overlap;
    }
    if (g->res_yend + overlap > kYGrid) {
        g->in_yend = kYGrid;
        g->iny = fy + overlap + (kYGrid - g->res_yend);
        g->pole = true;
    } else {
        g->in_yend = g->res_yend + overlap;
    }
    return true;
}

// global x (1-based) of local input column lx (1-based): tileoverlapgrid4d's
// periodic wrap (res_domain.f90:380-399)
inline int input_x(const RegionGeom &g, int lx) {
    if (g.periodic && (g.res_xend > g.in_xend || g.in_xstart > g.res_xstart)) {
        const int nfirst = kXGrid - (g.in_xstart - 1);
        return lx <= nfirst ? g.in_xstart + lx - 1 : lx - nfirst;
    }
    return g.in_xstart + lx - 1;
}

// feedback length for the bottom level: atmo + logp + precip + [sst] + tisr
// (allocate_res_new, mod_reservoir.f90:104-170)
inline int region_ninp(const RegionGeom &g, bool sst) {
    const int in2d = g.inx * g.iny;
    return kVars * in2d * kZGrid + in2d + in2d + (sst ? in2d : 0) + in2d;
}

// processor_decomposition (res_domain.f90:31-62): the regions rank irank of numprocs
// owns -- a contiguous block of numregions/numprocs, and for ranks 1..left one of the
// `left` leftover regions at the end (0-based region numbers)
inline int processor_regions(int numregions, int numprocs, int irank, int *out) {
    const int per = numregions / numprocs, left = numregions % numprocs;
    int c = 0;
    for (int i = 0; i < per; ++i) out[c++] = per * irank + i;
    if (irank > 0 && irank <= left) out[c++] = numregions - left + irank - 1;
    return c;
}

// grid4d(4,96,48,8) column-major index, 0-based arguments
inline int g4(int v, int x, int y, int z) { return v + kVars * (x + kXGrid * (y + kYGrid * z)); }
inline int g2(int x, int y) { return x + kXGrid * y; }

}  // namespace sml

#define SML_HIP(expr)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return ::sml::fail(SML_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
    } while (0)

#define SML_REQUIRE(cond, ...)                                 \
    do {                                                       \
        if (!(cond)) return ::sml::fail(SML_ERR_ARG, __VA_ARGS__); \
    } while (0)
