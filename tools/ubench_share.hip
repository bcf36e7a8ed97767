// Micro-benchmark: what do the waves of one CU share?  W waves (one workgroup of 64 W threads, one wave per SIMD)
// each run the same instruction stream; cycles per operation per wave (s_memtime) for W = 1, 2, 4.  A stream whose
// per-wave cost grows with W uses a per-CU shared resource.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_share tools/ubench_share.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int REP = 256;

// 4 independent f64 FMA chains
__global__ void k_fma4(double *out, unsigned long long *cyc, double a, double b)
{
    double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i) {
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x0) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x1) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x2) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x3) : "v"(a), "v"(b));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
}

// 4 independent v_rcp_f64 chains (transcendental)
__global__ void k_rcp4(double *out, unsigned long long *cyc)
{
    double x0 = 1.5 + threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i) {
        asm volatile("v_rcp_f64 %0, %0" : "+v"(x0));
        asm volatile("v_rcp_f64 %0, %0" : "+v"(x1));
        asm volatile("v_rcp_f64 %0, %0" : "+v"(x2));
        asm volatile("v_rcp_f64 %0, %0" : "+v"(x3));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
}

// independent ds_read_b64 (8 in flight, conflict-free consecutive addresses), then a wait
__global__ void k_lds64(double *out, unsigned long long *cyc)
{
    __shared__ double buf[8][64 * 8];
    const int w = threadIdx.x / 64, l = threadIdx.x & 63;
    for (int e = l; e < 64 * 8; e += 64) buf[w][e] = e;
    __syncthreads();
    double acc = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP / 8; ++i) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = buf[w][j * 64 + ((l + i) & 63)];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += v[j];
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

// independent ds_read_b128
__global__ void k_lds128(double *out, unsigned long long *cyc)
{
    typedef double d2 __attribute__((ext_vector_type(2)));
    __shared__ d2 buf[8][64 * 8];
    const int w = threadIdx.x / 64, l = threadIdx.x & 63;
    for (int e = l; e < 64 * 8; e += 64) buf[w][e] = d2{(double)e, 1.0};
    __syncthreads();
    double acc = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP / 8; ++i) {
        d2 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = buf[w][j * 64 + ((l + i) & 63)];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += v[j].x + v[j].y;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

// dependent LDS round trips (address from the previous read): latency
__global__ void k_ldsdep(double *out, unsigned long long *cyc)
{
    __shared__ int nxt[8][64 * 4];
    const int w = threadIdx.x / 64, l = threadIdx.x & 63;
    for (int e = l; e < 64 * 4; e += 64) nxt[w][e] = (e + 64 + 1) % (64 * 4);
    __syncthreads();
    int p = l;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
    for (int i = 0; i < REP; ++i) p = nxt[w][p];
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = p;
    if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}


// 8 independent 32-bit integer VALU chains (full-rate instructions: issue-bound)
__global__ void k_iadd8(double *out, unsigned long long *cyc)
{
    int x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_add_u32 %0, %0, 3" : "+v"(x[j]));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
}

// 8 independent SALU chains
__global__ void k_salu8(double *out, unsigned long long *cyc)
{
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
        "s_mov_b32 s40, 1\n s_mov_b32 s41, 2\n s_mov_b32 s42, 3\n s_mov_b32 s43, 4\n"
        "s_mov_b32 s44, 5\n s_mov_b32 s45, 6\n s_mov_b32 s46, 7\n s_mov_b32 s47, 8\n"
        ".rept 256\n s_add_u32 s40, s40, 3\n s_add_u32 s41, s41, 3\n s_add_u32 s42, s42, 3\n s_add_u32 s43, s43, 3\n"
        " s_add_u32 s44, s44, 3\n s_add_u32 s45, s45, 3\n s_add_u32 s46, s46, 3\n s_add_u32 s47, s47, 3\n .endr\n"
        ::: "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "scc");
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = 0;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
}

// 8 independent v_mov_b64 / v_cndmask-style 32-bit moves mixed with f64 FMAs (1 fma : 3 cheap)
__global__ void k_mix(double *out, unsigned long long *cyc, double a, double b)
{
    double x0 = threadIdx.x * 1e-3, x1 = x0 + 1;
    int y0 = threadIdx.x, y1 = y0 + 1, y2 = y0 + 2, y3 = y0 + 3, y4 = y0 + 4, y5 = y0 + 5;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i) {
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x0) : "v"(a), "v"(b));
        asm volatile("v_add_u32 %0, %0, 3" : "+v"(y0));
        asm volatile("v_add_u32 %0, %0, 3" : "+v"(y1));
        asm volatile("v_add_u32 %0, %0, 3" : "+v"(y2));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x1) : "v"(a), "v"(b));
        asm volatile("v_add_u32 %0, %0, 3" : "+v"(y3));
        asm volatile("v_add_u32 %0, %0, 3" : "+v"(y4));
        asm volatile("v_add_u32 %0, %0, 3" : "+v"(y5));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + y0 + y1 + y2 + y3 + y4 + y5;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
}

typedef void (*K0)(double *, unsigned long long *);

static double run(const char *name, int W, int ops, void (*launch)(int, double *, unsigned long long *),
                  double *dout, unsigned long long *dcyc, int nblk)
{
    hipMemset(dcyc, 0, nblk * 8 * sizeof(unsigned long long));
    launch(W, dout, dcyc);
    hipDeviceSynchronize();
    launch(W, dout, dcyc);
    hipDeviceSynchronize();
    unsigned long long h[1024 * 8];
    hipMemcpy(h, dcyc, nblk * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double s = 0;
    int n = 0;
    for (int b = 0; b < nblk; ++b)
        for (int w = 0; w < W; ++w) { s += (double)h[b * 8 + w]; n++; }
    const double c = s / n / ops;
    printf("%-10s W=%d  cycles/op per wave %.2f\n", name, W, c);
    return c;
}

int main()
{
    const int nblk = 256;   // about one workgroup per CU
    double *dout;
    unsigned long long *dcyc;
    hipMalloc(&dout, nblk * 512 * sizeof(double));
    hipMalloc(&dcyc, nblk * 8 * sizeof(unsigned long long));
    for (int W : {1, 2, 4, 8}) {
        run("fma4", W, REP * 4, [](int W, double *o, unsigned long long *c) {
            hipLaunchKernelGGL(k_fma4, dim3(256), dim3(64 * W), 0, 0, o, c, 1.0000001, 1e-9); }, dout, dcyc, nblk);
        run("rcp4", W, REP * 4, [](int W, double *o, unsigned long long *c) {
            hipLaunchKernelGGL(k_rcp4, dim3(256), dim3(64 * W), 0, 0, o, c); }, dout, dcyc, nblk);
        run("lds_b64", W, REP, [](int W, double *o, unsigned long long *c) {
            hipLaunchKernelGGL(k_lds64, dim3(256), dim3(64 * W), 0, 0, o, c); }, dout, dcyc, nblk);
        run("lds_b128", W, REP, [](int W, double *o, unsigned long long *c) {
            hipLaunchKernelGGL(k_lds128, dim3(256), dim3(64 * W), 0, 0, o, c); }, dout, dcyc, nblk);
        run("lds_dep", W, REP, [](int W, double *o, unsigned long long *c) {
            hipLaunchKernelGGL(k_ldsdep, dim3(256), dim3(64 * W), 0, 0, o, c); }, dout, dcyc, nblk);
        run("iadd8", W, REP * 8, [](int W, double *o, unsigned long long *c) {
            hipLaunchKernelGGL(k_iadd8, dim3(256), dim3(64 * W), 0, 0, o, c); }, dout, dcyc, nblk);
        run("salu8", W, 256 * 8, [](int W, double *o, unsigned long long *c) {
            hipLaunchKernelGGL(k_salu8, dim3(256), dim3(64 * W), 0, 0, o, c); }, dout, dcyc, nblk);
        run("mix(1:3)", W, REP * 8, [](int W, double *o, unsigned long long *c) {
            hipLaunchKernelGGL(k_mix, dim3(256), dim3(64 * W), 0, 0, o, c, 1.0000001, 1e-9); }, dout, dcyc, nblk);
    }
    hipFree(dout);
    hipFree(dcyc);
    return 0;
}
