// sml_spectral_tables.hpp -- T30 spectral operator tables built on the host.
#pragma once
#include "sml_internal.hpp"

namespace sml {

constexpr int kMX = 31, kNX = 32, kMX2 = 62, kIX = 96, kIY = 24, kIL = 48;
constexpr int kNTRUN = 30, kNTRUN1 = 31;
constexpr int kCPad = 64;  // Fourier-coefficient axis padded to the MFMA K granule

struct SpectralTables {
    double radius;
    double sia[kIY], wt[kIY], coa[kIY];
    double cosgr[kIL], cosgr2[kIL];
    int nsh2[kNX];
    double el2[kNX][kMX];
    double gradx[kMX];
    double gradym[kNX][kMX], gradyp[kNX][kMX];
    double uvdx[kNX][kMX], uvdym[kNX][kMX], uvdyp[kNX][kMX];
    double vddym[kNX][kMX], vddyp[kNX][kMX];
    double poly[kIY][kNX][kMX];   // P_mn at sia(j) (lgndre)
    double dinv[kCPad][kIX];      // inverse real-DFT matrix, coefficient c -> longitude i
    double dfwd[kIX][kCPad];      // forward real-DFT matrix, longitude i -> coefficient c
};

void build_spectral_tables(double radius, SpectralTables *t);

}  // namespace sml
