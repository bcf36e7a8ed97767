// Micro-benchmark + layout check for the f64 MFMA Riccati stage (gfx950), one wave, s_memtime cycles.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_mfma tools/ubench_mfma.hip
// (1) layout: v_mfma_f64_16x16x4_f64 with A lane l = A[l&15][k=l>>4], B lane l = B[k=l>>4][l&15],
//     D reg r of lane l = D[row 4r + (l>>4)][col l&15]; checked on exact integer data, including the chained
//     products W = P G (P's D layout as A, G as B) and M = G^T W (G's B registers as A, W's D layout as B).
// (2) timing: the 4-MFMA product, two chained products, an MFMA chain with independent / dependent f64 VALU work
//     interleaved (does the matrix unit run beside the VALU in one wave?), at 1 wave and at 4 waves per CU.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int REP = 128;

__device__ inline d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

// ---- (1) layout ------------------------------------------------------------------------------------------
// in: P (16x16, symmetric), G (16x16), Out: W = P G, M = G^T W (row-major 16x16 each)
__global__ void k_layout(const double *P, const double *G, double *W, double *M, double *D1, const double *A1,
                         const double *B1)
{
    const int l = threadIdx.x, c = l & 15, g = l >> 4;
    // single 16x16x4: D1 = A1 (16x4) * B1 (4x16)
    d4 z = {0, 0, 0, 0};
    d4 d1 = mfma(A1[c * 4 + g], B1[g * 16 + c], z);
    for (int r = 0; r < 4; ++r) D1[(4 * r + g) * 16 + c] = d1[r];
    // P in D layout (reg s: P[4s+g][c]), G in B layout (reg s: G[4s+g][c])
    double p[4], gb[4];
    for (int s = 0; s < 4; ++s) {
        p[s] = P[(4 * s + g) * 16 + c];
        gb[s] = G[(4 * s + g) * 16 + c];
    }
    d4 w = z;
    for (int s = 0; s < 4; ++s) w = mfma(p[s], gb[s], w);   // A = P (via symmetry), B = G
    d4 m = z;
    for (int s = 0; s < 4; ++s) m = mfma(gb[s], w[s], m);   // A = G^T, B = W
    for (int r = 0; r < 4; ++r) {
        W[(4 * r + g) * 16 + c] = w[r];
        M[(4 * r + g) * 16 + c] = m[r];
    }
}

// ---- (2) timing --------------------------------------------------------------------------------------------
// product chain: X <- X G (4 MFMAs, X's D layout used as the next A operand), NP times
__global__ void k_prod_chain(double *out, unsigned long long *cyc, double gv, int np)
{
    const int l = threadIdx.x;
    d4 x = {l * 1e-3, 1.0, 0.5, 0.25};
    const double g0 = gv, g1 = gv * 0.5, g2 = gv * 0.25, g3 = gv * 0.125;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < np; ++i) {
        d4 y = {0, 0, 0, 0};
        y = mfma(x[0], g0, y);
        y = mfma(x[1], g1, y);
        y = mfma(x[2], g2, y);
        y = mfma(x[3], g3, y);
        x = y;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + l] = x[0] + x[1] + x[2] + x[3];
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// W = P G then M = G^T W (8 MFMAs, the stage pair) then P <- M (repeat): the stage's MFMA critical path
__global__ void k_stage_pair(double *out, unsigned long long *cyc, double gv, int np)
{
    const int l = threadIdx.x;
    d4 p = {l * 1e-3, 1.0, 0.5, 0.25};
    const double g[4] = {gv, gv * 0.5, gv * 0.25, gv * 0.125};
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < np; ++i) {
        d4 w = {0, 0, 0, 0}, m = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < 4; ++s) w = mfma(p[s], g[s], w);
#pragma unroll
        for (int s = 0; s < 4; ++s) m = mfma(g[s], w[s], m);
        p = m;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + l] = p[0] + p[1] + p[2] + p[3];
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// MFMA accumulate chain with NV independent v_fma_f64 per MFMA (asm keeps the interleave)
template <int NV>
__global__ void k_mfma_valu_ind(double *out, unsigned long long *cyc, double a, double b)
{
    const int l = threadIdx.x;
    d4 acc = {l * 1e-3, 0.0, 0.0, 0.0};
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = l * 1e-3 + j;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
    for (int i = 0; i < REP; ++i) {
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
#pragma unroll
        for (int j = 0; j < NV; ++j) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v[j & 7]) : "v"(a), "v"(b));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = acc[0] + acc[1] + acc[2] + acc[3];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
    out[blockIdx.x * 64 + l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// the same VALU work alone (reference)
template <int NV>
__global__ void k_valu_ind(double *out, unsigned long long *cyc, double a, double b)
{
    const int l = threadIdx.x;
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = l * 1e-3 + j;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
    for (int i = 0; i < REP; ++i) {
#pragma unroll
        for (int j = 0; j < NV; ++j) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v[j & 7]) : "v"(a), "v"(b));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
    out[blockIdx.x * 64 + l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// MFMA accumulate chain with a dependent v_fma_f64 chain of ND per MFMA
template <int ND>
__global__ void k_mfma_valu_dep(double *out, unsigned long long *cyc, double a, double b)
{
    const int l = threadIdx.x;
    d4 acc = {l * 1e-3, 0.0, 0.0, 0.0};
    double v = l * 1e-3;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
    for (int i = 0; i < REP; ++i) {
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
#pragma unroll
        for (int j = 0; j < ND; ++j) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v) : "v"(a), "v"(b));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + l] = acc[0] + acc[1] + acc[2] + acc[3] + v;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}


// MFMA accumulate chain with NV independent 32-bit integer VALU ops per MFMA (v_add_u32): does non-FP64 VALU work
// issue while the matrix core holds the FP64 pipeline?
template <int NV>
__global__ void k_mfma_int(double *out, unsigned long long *cyc, double a, double b)
{
    const int l = threadIdx.x;
    d4 acc = {l * 1e-3, 0.0, 0.0, 0.0};
    unsigned v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = l + j;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
    for (int i = 0; i < REP; ++i) {
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
#pragma unroll
        for (int j = 0; j < NV; ++j) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[j & 7]) : "v"(l));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
    out[blockIdx.x * 64 + l] = acc[0] + acc[1] + acc[2] + acc[3] + s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int NV>
__global__ void k_int_alone(double *out, unsigned long long *cyc)
{
    const int l = threadIdx.x;
    unsigned v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = l + j;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
    for (int i = 0; i < REP; ++i) {
#pragma unroll
        for (int j = 0; j < NV; ++j) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[j & 7]) : "v"(l));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
    out[blockIdx.x * 64 + l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}
// MFMA chain with NV independent ds_read_b64 per MFMA (results kept alive)
template <int NV>
__global__ void k_mfma_lds(double *out, unsigned long long *cyc, double a, double b)
{
    __shared__ double buf[1024];
    const int l = threadIdx.x;
    for (int j = l; j < 1024; j += 64) buf[j] = j;
    __syncthreads();
    d4 acc = {l * 1e-3, 0.0, 0.0, 0.0};
    double r[8];
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
    for (int i = 0; i < REP; ++i) {
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
#pragma unroll
        for (int j = 0; j < NV; ++j) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r[j & 7]) : "v"(l * 8), "i"(j * 512));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += (j < NV) ? r[j] : 0.0;
    out[blockIdx.x * 64 + l] = acc[0] + acc[1] + acc[2] + acc[3] + s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// cross-lane: sum over the four 16-lane groups with permlane16/32 swaps (f64 = two dwords each), dependent chain
__device__ inline double grp4_sum(double v)
{
    long long b = __double_as_longlong(v);
    int lo = (int)b, hi = (int)(b >> 32);
    auto r0 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto r1 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    double a0 = __longlong_as_double(((long long)(unsigned)r1[0] << 32) | (unsigned)r0[0]);
    double a1 = __longlong_as_double(((long long)(unsigned)r1[1] << 32) | (unsigned)r0[1]);
    double s = a0 + a1;
    b = __double_as_longlong(s);
    lo = (int)b;
    hi = (int)(b >> 32);
    auto q0 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto q1 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    double c0 = __longlong_as_double(((long long)(unsigned)q1[0] << 32) | (unsigned)q0[0]);
    double c1 = __longlong_as_double(((long long)(unsigned)q1[1] << 32) | (unsigned)q0[1]);
    return c0 + c1;
}
__global__ void k_grp4(double *out, unsigned long long *cyc, const double *in)
{
    const int l = threadIdx.x;
    double v = in[l];
    out[64 + l] = grp4_sum(v);   // correctness
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) v = grp4_sum(v) * 0.25;
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[l] = v;
    if (l == 0) cyc[0] = t1 - t0;
}

int main()
{
    // ---- layout check
    double hP[256], hG[256], hA1[64], hB1[64];
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            hP[i * 16 + j] = (double)((i + 1) * (j + 1) % 7 + (i == j ? 3 : 0));   // symmetric
            hG[i * 16 + j] = (double)((3 * i + 5 * j) % 11 - 5);                      // asymmetric
        }
    for (int i = 0; i < 16; ++i)
        for (int k = 0; k < 4; ++k) hA1[i * 4 + k] = (double)(i * 4 + k + 1);
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 16; ++j) hB1[k * 16 + j] = (double)((k + 2) * (j + 1) % 13 - 6);
    double *dP, *dG, *dW, *dM, *dD1, *dA1, *dB1;
    hipMalloc(&dP, 2048); hipMalloc(&dG, 2048); hipMalloc(&dW, 2048); hipMalloc(&dM, 2048);
    hipMalloc(&dD1, 2048); hipMalloc(&dA1, 512); hipMalloc(&dB1, 512);
    hipMemcpy(dP, hP, 2048, hipMemcpyHostToDevice);
    hipMemcpy(dG, hG, 2048, hipMemcpyHostToDevice);
    hipMemcpy(dA1, hA1, 512, hipMemcpyHostToDevice);
    hipMemcpy(dB1, hB1, 512, hipMemcpyHostToDevice);
    k_layout<<<1, 64>>>(dP, dG, dW, dM, dD1, dA1, dB1);
    double hW[256], hM[256], hD1[256];
    hipMemcpy(hW, dW, 2048, hipMemcpyDeviceToHost);
    hipMemcpy(hM, dM, 2048, hipMemcpyDeviceToHost);
    hipMemcpy(hD1, dD1, 2048, hipMemcpyDeviceToHost);
    int bad1 = 0, badW = 0, badM = 0;
    double rW[256], rM[256];
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double d = 0, w = 0;
            for (int k = 0; k < 4; ++k) d += hA1[i * 4 + k] * hB1[k * 16 + j];
            for (int k = 0; k < 16; ++k) w += hP[i * 16 + k] * hG[k * 16 + j];
            rW[i * 16 + j] = w;
            bad1 += d != hD1[i * 16 + j];
            badW += w != hW[i * 16 + j];
        }
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double m = 0;
            for (int k = 0; k < 16; ++k) m += hG[k * 16 + i] * rW[k * 16 + j];
            rM[i * 16 + j] = m;
            badM += m != hM[i * 16 + j];
        }
    printf("layout: single 16x16x4 mismatches %d/256, W = P G %d/256, M = G^T W %d/256\n", bad1, badW, badM);

    // ---- timing
    double *out;
    unsigned long long *cyc, h[1024];
    hipMalloc(&out, 1024 * 64 * 16 * sizeof(double));
    hipMalloc(&cyc, 1024 * sizeof(unsigned long long));
    auto run = [&](const char *name, auto launch, int nblk, double ops) {
        for (int w = 0; w < 3; ++w) launch();
        hipDeviceSynchronize();
        launch();
        hipDeviceSynchronize();
        hipMemcpy(h, cyc, nblk * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        double mean = 0, mx = 0;
        for (int b = 0; b < nblk; ++b) {
            mean += (double)h[b] / nblk;
            mx = fmax(mx, (double)h[b]);
        }
        printf("%-44s grid %4d: %8.2f cycles/op (mean), %8.2f (max)\n", name, nblk, mean / ops, mx / ops);
    };
    for (int nb : {1, 1024}) {
        run("product X <- X G (4 mfma) chain", [&] { k_prod_chain<<<nb, 64>>>(out, cyc, 0.999, REP); }, nb, REP);
        run("stage pair W=PG, M=G^T W (8 mfma)", [&] { k_stage_pair<<<nb, 64>>>(out, cyc, 0.999, REP); }, nb, REP);
        run("mfma chain alone (per mfma)", [&] { k_mfma_valu_ind<0><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
        run("mfma + 4 ind fma (per mfma)", [&] { k_mfma_valu_ind<4><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
        run("mfma + 8 ind fma (per mfma)", [&] { k_mfma_valu_ind<8><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
        run("mfma + 16 ind fma (per mfma)", [&] { k_mfma_valu_ind<16><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
        run("16 ind fma alone (per group)", [&] { k_valu_ind<16><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
        run("mfma + 4 dep fma (per mfma)", [&] { k_mfma_valu_dep<4><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
        run("mfma + 6 dep fma (per mfma)", [&] { k_mfma_valu_dep<6><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
        run("mfma + 12 dep fma (per mfma)", [&] { k_mfma_valu_dep<12><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
        run("mfma + 8 ind v_add_u32 (per mfma)", [&] { k_mfma_int<8><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
        run("mfma + 16 ind v_add_u32 (per mfma)", [&] { k_mfma_int<16><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
        run("16 ind v_add_u32 alone (per group)", [&] { k_int_alone<16><<<nb, 64>>>(out, cyc); }, nb, REP);
        run("mfma + 4 ds_read_b64 + wait (per mfma)", [&] { k_mfma_lds<4><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
        run("mfma + 8 ds_read_b64 + wait (per mfma)", [&] { k_mfma_lds<8><<<nb, 64>>>(out, cyc, 0.999, 1e-3); }, nb, REP);
    }
    {
        double hin[64], hout[128];
        for (int l = 0; l < 64; ++l) hin[l] = l + 1;
        double *din;
        hipMalloc(&din, 512);
        hipMemcpy(din, hin, 512, hipMemcpyHostToDevice);
        run("grp4_sum (permlane32+16 swaps) dependent", [&] { k_grp4<<<1, 64>>>(out, cyc, din); }, 1, REP);
        hipMemcpy(hout, out, 1024, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; ++l) {
            const int c = l & 15;
            bad += hout[64 + l] != (hin[c] + hin[c + 16] + hin[c + 32] + hin[c + 48]);
        }
        printf("grp4_sum mismatches %d/64\n", bad);
    }
    return 0;
}
