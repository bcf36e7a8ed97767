// Micro-benchmark: per-instruction latency / issue cost on one wave (gfx950), measured with s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_latency tools/ubench_latency.hip
// Prints cycles per operation for: dependent FP64 FMA chain, 4 interleaved chains, v_rsq_f64 chain,
// dependent LDS read chain, back-to-back global stores (issue cost), ds_write_b64 issue and f64 MFMA 16x16x4.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int REP = 256;

__global__ void k_fma_dep(double *out, unsigned long long *cyc, double a, double b)
{
    double x = threadIdx.x * 1e-3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_fma_ind4(double *out, unsigned long long *cyc, double a, double b)
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
    out[threadIdx.x] = x0 + x1 + x2 + x3;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_mul_dep(double *out, unsigned long long *cyc, double a)
{
    double x = threadIdx.x * 1e-3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x) : "v"(a));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_fma_f32_dep(double *out, unsigned long long *cyc, float a, float b)
{
    float x = threadIdx.x * 1e-3f;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_rsq_dep(double *out, unsigned long long *cyc)
{
    double x = 1.0 + threadIdx.x * 1e-3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i) asm volatile("v_rsq_f64 %0, %0" : "+v"(x));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_lds_dep(double *out, unsigned long long *cyc)
{
    __shared__ int nxt[64];
    nxt[threadIdx.x] = (threadIdx.x + 1) & 63;
    __syncthreads();
    int p = threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i) p = nxt[p];
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = p;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// issue cost of global stores: REP stores to distinct addresses, time until the last one is issued
__global__ void k_gstore(double *out, unsigned long long *cyc, int active)
{
    double v = threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if ((int)threadIdx.x < active) {
#pragma unroll
        for (int i = 0; i < REP; ++i) out[1024 + i * 64 + threadIdx.x] = v + i;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// the same stores followed by a full drain (vmcnt(0)): completion latency
__global__ void k_gstore_drain(double *out, unsigned long long *cyc)
{
    double v = threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < 16; ++i) out[1024 + i * 64 + threadIdx.x] = v + i;
    __builtin_amdgcn_s_waitcnt(0);   // vmcnt(0) expcnt(0) lgkmcnt(0)
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_dswrite(double *out, unsigned long long *cyc)
{
    __shared__ double buf[64 * 8];
    double v = threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i) buf[(i & 7) * 64 + threadIdx.x] = v + i;
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    out[threadIdx.x] = buf[threadIdx.x];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// f64 MFMA (the Riccati contractions' candidate unit): one V_MFMA_F64_16X16X4_F64 chain on its
// accumulator, and four independent accumulators (cycles per MFMA)
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k_mfma_dep(double *out, unsigned long long *cyc, double a, double b)
{
    d4 acc = {threadIdx.x * 1e-3, 0.0, 0.0, 0.0};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_mfma_ind4(double *out, unsigned long long *cyc, double a, double b)
{
    d4 c0 = {threadIdx.x * 1e-3, 0.0, 0.0, 0.0}, c1 = c0, c2 = c0, c3 = c0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; ++i) {
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c1) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c2) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c3) : "v"(a), "v"(b));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main()
{
    double *out;
    unsigned long long *cyc, h;
    hipMalloc(&out, (1024 + REP * 64) * sizeof(double));
    hipMalloc(&cyc, sizeof(unsigned long long));
    auto run = [&](const char *name, auto launch, int ops) {
        for (int w = 0; w < 3; ++w) launch();   // warm (code fetch, clocks)
        hipDeviceSynchronize();
        launch();
        hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        printf("%-28s %8.2f cycles/op  (%llu over %d)\n", name, (double)h / ops, h, ops);
    };
    run("fma_f64 dependent", [&] { k_fma_dep<<<1, 64>>>(out, cyc, 0.999, 1e-3); }, REP);
    run("fma_f64 4 chains (per fma)", [&] { k_fma_ind4<<<1, 64>>>(out, cyc, 0.999, 1e-3); }, 4 * REP);
    run("mul_f64 dependent", [&] { k_mul_dep<<<1, 64>>>(out, cyc, 0.999); }, REP);
    run("fma_f32 dependent", [&] { k_fma_f32_dep<<<1, 64>>>(out, cyc, 0.999f, 1e-3f); }, REP);
    run("rsq_f64 dependent", [&] { k_rsq_dep<<<1, 64>>>(out, cyc); }, REP);
    run("ds_read_b32 dependent", [&] { k_lds_dep<<<1, 64>>>(out, cyc); }, REP);
    run("global_store x2 issue 64L", [&] { k_gstore<<<1, 64>>>(out, cyc, 64); }, REP);
    run("global_store x2 issue 17L", [&] { k_gstore<<<1, 64>>>(out, cyc, 17); }, REP);
    run("16 stores + drain (total)", [&] { k_gstore_drain<<<1, 64>>>(out, cyc); }, 1);
    run("ds_write_b64 issue", [&] { k_dswrite<<<1, 64>>>(out, cyc); }, REP);
    run("mfma_f64_16x16x4 dependent", [&] { k_mfma_dep<<<1, 64>>>(out, cyc, 0.999, 1e-3); }, REP);
    run("mfma_f64_16x16x4 4 chains", [&] { k_mfma_ind4<<<1, 64>>>(out, cyc, 0.999, 1e-3); }, 4 * REP);
    hipFree(out);
    hipFree(cyc);
    return 0;
}
