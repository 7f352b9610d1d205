// Operand / result lane layout of v_mfma_f64_4x4x4_f64 (4 blocks of 4x4x4), found by
// indicator products: for every (A lane ja, B lane jb) pair, A = 1 only on lane ja and
// B = 1 only on lane jb; the output lanes that come out 1 hold C[m][n] with A[m][k] on
// ja and B[k][n] on jb.  Prints, per output lane, the (ja, jb) pairs that reach it.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma44_layout tools/probe_mfma44_layout.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void k(double *out) {
    const int l = threadIdx.x;
    for (int ja = 0; ja < 64; ++ja)
        for (int jb = 0; jb < 64; ++jb) {
            const double a = l == ja ? 1.0 : 0.0, b = l == jb ? 1.0 : 0.0;
            const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
            out[((size_t)ja * 64 + jb) * 64 + l] = d;
        }
}

int main() {
    double *d;
    hipMalloc(&d, 64 * 64 * 64 * 8);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    std::vector<double> h(64 * 64 * 64);
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) {
        printf("out lane %2d:", l);
        for (int ja = 0; ja < 64; ++ja)
            for (int jb = 0; jb < 64; ++jb)
                if (h[((size_t)ja * 64 + jb) * 64 + l] != 0.0) printf(" (%d,%d)", ja, jb);
        printf("\n");
    }
    return 0;
}
