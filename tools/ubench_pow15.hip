// Device arithmetic check: mu^1.5 (ipm_kernel.hip pow15), fp64 sqrt and division on the values the solver's
// barrier update produces, written out for an exact comparison on the host (tools/check_pow15.py).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_pow15 tools/ubench_pow15.hip && ./tools/ubench_pow15 out.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

__device__ inline double pow15(double x)
{
#ifndef CONTRACT
#pragma clang fp contract(off)
#endif
    const double s = sqrt(x);
    const double slo = fma(-s, s, x) / (2.0 * s);
    const double p = x * s;
    const double plo = fma(x, s, -p);
    return p + fma(x, slo, plo);
}

__global__ void k(const double *x, double *out, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    const double s = sqrt(v);
    out[4 * i + 0] = pow15(v);
    out[4 * i + 1] = s;
    out[4 * i + 2] = fma(-s, s, v) / (2.0 * s);
    out[4 * i + 3] = v / 3.0;
}

int main(int argc, char **argv)
{
    const int n = 4096;
    std::vector<double> x(n);
    unsigned long long r = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        r ^= r << 13; r ^= r >> 7; r ^= r << 17;
        x[i] = std::pow(10.0, -9.0 + 9.0 * (double)(r >> 11) / 9007199254740992.0);
    }
    x[0] = 1.5042412372345582e-4; x[1] = 0.020000000000000004; x[2] = 0.1;
    double *dx, *dout;
    if (hipMalloc(&dx, n * 8) != hipSuccess || hipMalloc(&dout, 4 * n * 8) != hipSuccess) return 1;
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dout, n);
    std::vector<double> out(4 * n);
    if (hipMemcpy(out.data(), dout, 4 * n * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    FILE *f = fopen(argc > 1 ? argv[1] : "pow15.bin", "wb");
    fwrite(x.data(), 8, n, f);
    fwrite(out.data(), 8, 4 * n, f);
    fclose(f);
    printf("wrote %d values\n", n);
    return 0;
}
