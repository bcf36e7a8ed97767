// Micro-benchmark: LDS read throughput per CU as the Riccati stage uses it.  W waves per CU (one workgroup of
// 64 W threads, one wave per SIMD), each issuing batches of 8 independent ds_read_b128 / ds_read_b64 (waited
// per batch, consumed by integer xors), with ACT of the 64 lanes active (exec mask) and per-lane distinct or
// wave-uniform (broadcast) addresses.  Cycles per read instruction per wave (s_memtime) tell whether inactive
// lanes and broadcast reads cost LDS bandwidth.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_lds tools/ubench_lds.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int REP = 64;   // batches of 8 reads

template <int B128, int BCAST>
__global__ void k_lds(unsigned *out, unsigned long long *cyc, int act)
{
    __shared__ __attribute__((aligned(16))) double buf[8][8 * 64 * 2];
    const int w = threadIdx.x / 64, l = threadIdx.x & 63;
    for (int e = l; e < 8 * 64 * 2; e += 64) buf[w][e] = (double)e;
    __syncthreads();
    unsigned acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned base = (unsigned)(size_t)&buf[w][0];
    const unsigned la = BCAST ? 0u : (unsigned)l * (B128 ? 16u : 8u);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (l < act) {
        for (int i = 0; i < REP; ++i) {
            const unsigned a = base + la;
            if (B128) {
                typedef unsigned u4 __attribute__((ext_vector_type(4)));
                u4 v0, v1, v2, v3, v4, v5, v6, v7;
                asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(v0) : "v"(a));
                asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(v1) : "v"(a));
                asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(v2) : "v"(a));
                asm volatile("ds_read_b128 %0, %1 offset:3072" : "=v"(v3) : "v"(a));
                asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(v4) : "v"(a));
                asm volatile("ds_read_b128 %0, %1 offset:5120" : "=v"(v5) : "v"(a));
                asm volatile("ds_read_b128 %0, %1 offset:6144" : "=v"(v6) : "v"(a));
                asm volatile("ds_read_b128 %0, %1 offset:7168" : "=v"(v7) : "v"(a));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                acc[0] ^= v0.x; acc[1] ^= v1.x; acc[2] ^= v2.x; acc[3] ^= v3.x;
                acc[4] ^= v4.x; acc[5] ^= v5.x; acc[6] ^= v6.x; acc[7] ^= v7.x;
            } else {
                typedef unsigned u2 __attribute__((ext_vector_type(2)));
                u2 v0, v1, v2, v3, v4, v5, v6, v7;
                asm volatile("ds_read_b64 %0, %1 offset:0" : "=v"(v0) : "v"(a));
                asm volatile("ds_read_b64 %0, %1 offset:512" : "=v"(v1) : "v"(a));
                asm volatile("ds_read_b64 %0, %1 offset:1024" : "=v"(v2) : "v"(a));
                asm volatile("ds_read_b64 %0, %1 offset:1536" : "=v"(v3) : "v"(a));
                asm volatile("ds_read_b64 %0, %1 offset:2048" : "=v"(v4) : "v"(a));
                asm volatile("ds_read_b64 %0, %1 offset:2560" : "=v"(v5) : "v"(a));
                asm volatile("ds_read_b64 %0, %1 offset:3072" : "=v"(v6) : "v"(a));
                asm volatile("ds_read_b64 %0, %1 offset:3584" : "=v"(v7) : "v"(a));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                acc[0] ^= v0.x; acc[1] ^= v1.x; acc[2] ^= v2.x; acc[3] ^= v3.x;
                acc[4] ^= v4.x; acc[5] ^= v5.x; acc[6] ^= v6.x; acc[7] ^= v7.x;
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s ^= acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

template <int B128, int BCAST>
static void run(const char *name, int W, int act, unsigned *dout, unsigned long long *dcyc, int nblk)
{
    for (int r = 0; r < 2; ++r) {
        hipLaunchKernelGGL((k_lds<B128, BCAST>), dim3(nblk), dim3(64 * W), 0, 0, dout, dcyc, act);
        hipDeviceSynchronize();
    }
    unsigned long long h[1024 * 8];
    hipMemcpy(h, dcyc, nblk * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double s = 0;
    int n = 0;
    for (int b = 0; b < nblk; ++b)
        for (int w = 0; w < W; ++w) { s += (double)h[b * 8 + w]; n++; }
    printf("%-14s W=%d act=%2d  cycles/read per wave %.2f\n", name, W, act, s / n / (REP * 8));
}

int main()
{
    const int nblk = 256;
    unsigned *dout;
    unsigned long long *dcyc;
    hipMalloc(&dout, nblk * 512 * sizeof(unsigned));
    hipMalloc(&dcyc, nblk * 8 * sizeof(unsigned long long));
    for (int W : {1, 4, 8})
        for (int act : {64, 32, 17}) {
            run<1, 0>("b128 distinct", W, act, dout, dcyc, nblk);
            run<1, 1>("b128 bcast", W, act, dout, dcyc, nblk);
            run<0, 0>("b64 distinct", W, act, dout, dcyc, nblk);
            run<0, 1>("b64 bcast", W, act, dout, dcyc, nblk);
        }
    hipFree(dout);
    hipFree(dcyc);
    return 0;
}
