// moving.hip — traversal-time fixed point of the moving-gate loop (included by api.hip).
//
// quad_moving.py:29-57 (solver) for B episodes in one launch: t1 = |centroid(gate) - r| / 3, then
//   t2 = DNN2(inputs of the gate advanced by velo t1 and pitched by w t1)[6],  t1 += (t2 - t1) / 2
// until |t2 - t1| <= 0.001 (at most 200 updates).  The 18 DNN2 inputs are main.py:90-94 / quad_moving.py:38-42
// (gate.rotate_y / translate / transform / t_final, quad_model.py:686-815, with scipy's Rotation conventions
// for the attitude: from_quat normalises, from_matrix picks the largest of the diagonal and the trace), in
// fp64 exactly as moving_gate.dnn2_inputs_t; DNN2 (18-128-128-7 ReLU MLP, nn3_1.pth) runs in fp32 as the
// reference's forward does, only the time output row 6 of the last layer being formed.
//
// One wave per episode (grid-stride over the episodes): lane l owns hidden units l and l + 64 of both layers,
// with its two rows of the second layer's weight (256 floats) and of the first (36) held in registers for the
// whole launch, so an evaluation is 2 x 18 + 2 x 128 FMAs per lane and one 512-byte exchange of the first
// layer's activations through LDS (read back as wave-wide broadcasts); the time output is a 64-lane
// reduction.  The fixed point and the fp64 input transform are wave-uniform: every episode converges on its
// own count of updates.  Replaces ~80 small torch kernels per fixed-point iteration on the device path
// (moving_gate.FixedPointGraph).
namespace lafse3 {

constexpr int TT_IN = 18, TT_H = 128;
// packed weights: W1 [128][18], b1, W2 [128][128] (l2.weight, row j = output unit), b2, l3.weight row 6, l3.bias[6]
constexpr int TT_W1 = 0, TT_B1 = TT_W1 + TT_H * TT_IN, TT_W2 = TT_B1 + TT_H, TT_B2 = TT_W2 + TT_H * TT_H;
constexpr int TT_W3 = TT_B2 + TT_H;   // row 6 of the last layer's weight (128), then its bias
constexpr int TT_NW = TT_W3 + TT_H + 1;
constexpr double TT_TOL = 0.001;      // quad_moving.py:45
constexpr int TT_MAXIT = 200;

struct TTArgs {
    int64_t B;
    const double *state, *final_point, *gate, *velo;   // B x 13, B x 3, B x 12 (4 corners), B x 3
    double w;                                           // gate pitch rate (main.py:46)
    const float *weights;                               // TT_NW floats (layout above)
    double *t_out;
    int32_t *iters;
};

__device__ inline void tt_cross(const double *a, const double *b, double *c)
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

// the 18 DNN2 inputs for gate corners g (already advanced), moving_gate.dnn2_inputs_t
__device__ inline void tt_inputs(const double *g, const double *st, const double *fin, double *in)
{
    double cen[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) cen[a] = ((g[a] + g[3 + a]) + g[6 + a] + g[9 + a]) / 4.0;
    double e1[3], e2[3], ay[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        e1[a] = g[3 + a] - g[a];
        e2[a] = g[6 + a] - g[3 + a];
    }
    tt_cross(e1, e2, ay);
    const double n = sqrt(ay[0] * ay[0] + ay[1] * ay[1] + ay[2] * ay[2]);
#pragma unroll
    for (int a = 0; a < 3; ++a) ay[a] = ay[a] / n;
    const double az[3] = {0.0, 0.0, 1.0};
    double ax[3];
    tt_cross(ay, az, ax);
    const double IG[3][3] = {{ax[0], ax[1], ax[2]}, {ay[0], ay[1], ay[2]}, {az[0], az[1], az[2]}};
    double dr[3], df[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        dr[a] = st[a] - cen[a];
        df[a] = fin[a] - cen[a];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        in[i] = IG[i][0] * dr[0] + IG[i][1] * dr[1] + IG[i][2] * dr[2];
        in[3 + i] = IG[i][0] * st[3] + IG[i][1] * st[4] + IG[i][2] * st[5];
        in[13 + i] = IG[i][0] * df[0] + IG[i][1] * df[1] + IG[i][2] * df[2];
    }
    // attitude: scipy from_quat ([x, y, z, w], normalised) -> matrix, IG R, from_matrix -> quaternion
    double x = st[7], y = st[8], z = st[9], w = st[6];
    const double qn = sqrt(x * x + y * y + z * z + w * w);
    x /= qn; y /= qn; z /= qn; w /= qn;
    const double x2 = x * x, y2 = y * y, z2 = z * z, w2 = w * w;
    const double xy = x * y, zw = z * w, xz = x * z, yw = y * w, yz = y * z, xw = x * w;
    const double R[3][3] = {{x2 - y2 - z2 + w2, 2 * (xy - zw), 2 * (xz + yw)},
                            {2 * (xy + zw), -x2 + y2 - z2 + w2, 2 * (yz - xw)},
                            {2 * (xz - yw), 2 * (yz + xw), -x2 - y2 + z2 + w2}};
    double m[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) m[i][j] = IG[i][0] * R[0][j] + IG[i][1] * R[1][j] + IG[i][2] * R[2][j];
    const double d[3] = {m[0][0], m[1][1], m[2][2]};
    const double tr = (d[0] + d[1]) + d[2];
    int choice = 0;   // argmax of [m00, m11, m22, trace], first maximum
    double best = d[0];
    if (d[1] > best) { best = d[1]; choice = 1; }
    if (d[2] > best) { best = d[2]; choice = 2; }
    if (tr > best) choice = 3;
    double q[4];
    if (choice == 3) {
        q[0] = m[2][1] - m[1][2];
        q[1] = m[0][2] - m[2][0];
        q[2] = m[1][0] - m[0][1];
        q[3] = 1 + tr;
    } else {
        const int i = choice, j = (i + 1) % 3, k = (i + 2) % 3;
        q[i] = 1 - tr + 2 * m[i][i];
        q[j] = m[j][i] + m[i][j];
        q[k] = m[k][i] + m[i][k];
        q[3] = m[k][j] - m[j][k];
    }
    const double nq = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    in[6] = q[3] / nq;
    in[7] = q[0] / nq;
    in[8] = q[1] / nq;
    in[9] = q[2] / nq;
    in[10] = st[10];
    in[11] = st[11];
    in[12] = st[12];
    double d01[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) d01[a] = g[a] - g[3 + a];
    in[16] = sqrt(d01[0] * d01[0] + d01[1] * d01[1] + d01[2] * d01[2]);
    in[17] = atan(d01[2] / d01[0]);
}


// DNN2's time output at the fp32 inputs x (wave-uniform): lane l forms h_l, h_{l+64} of the first layer, the
// 128 activations are exchanged through hs, lane l accumulates units l and l + 64 of the second layer in
// input order (i = 0..127, fma from the bias), and the last layer's row 6 is reduced across the wave.
struct TTLane {
    float w2a[TT_H], w2b[TT_H];     // l2.weight rows l, l + 64
    float w1a[TT_IN], w1b[TT_IN];   // l1.weight rows l, l + 64
    float b1a, b1b, b2a, b2b, w3a, w3b, b3;
};

__device__ inline float tt_dnn2_time(const TTLane &L, float *hs, const float *x)
{
    float a = L.b1a, b = L.b1b;
#pragma unroll
    for (int k = 0; k < TT_IN; ++k) {
        a = fmaf(L.w1a[k], x[k], a);
        b = fmaf(L.w1b[k], x[k], b);
    }
    const int l = threadIdx.x;
    __syncthreads();                 // the previous evaluation's reads of hs are done
    hs[l] = fmaxf(a, 0.0f);
    hs[l + 64] = fmaxf(b, 0.0f);
    __syncthreads();
    float acc_a = L.b2a, acc_b = L.b2b;
#pragma unroll
    for (int i = 0; i < TT_H; ++i) {
        const float h = hs[i];       // same address in every lane: broadcast (merged into 16-byte reads)
        acc_a = fmaf(L.w2a[i], h, acc_a);
        acc_b = fmaf(L.w2b[i], h, acc_b);
    }
    float o = L.w3a * fmaxf(acc_a, 0.0f) + L.w3b * fmaxf(acc_b, 0.0f);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) o += __shfl_xor(o, m, 64);
    return o + L.b3;
}

// t -> DNN2's time for the gate advanced to t (wave-uniform)
__device__ inline double tt_time_at(const TTLane &L, float *hs, const double *g0, const double *st,
                                    const double *fin, const double *velo, double w, double t)
{
    // gate.translate(velo t) then gate.rotate_y(w t) about its centroid (x-z plane)
    double g[12];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int a = 0; a < 3; ++a) g[3 * c + a] = g0[3 * c + a] + velo[a] * t;
    double cen[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) cen[a] = ((g[a] + g[3 + a]) + g[6 + a] + g[9 + a]) / 4.0;
    const double ang = w * t, ca = cos(ang), sa = sin(ang);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const double x0 = g[3 * c] - cen[0], y0 = g[3 * c + 1] - cen[1], z0 = g[3 * c + 2] - cen[2];
        g[3 * c] = (ca * x0 + (-sa) * z0) + cen[0];
        g[3 * c + 1] = y0 + cen[1];
        g[3 * c + 2] = (sa * x0 + ca * z0) + cen[2];
    }
    double in[TT_IN];
    tt_inputs(g, st, fin, in);
    float x[TT_IN];
#pragma unroll
    for (int k = 0; k < TT_IN; ++k) x[k] = (float)in[k];
    return (double)tt_dnn2_time(L, hs, x);
}

__global__ __launch_bounds__(64) void traversal_time_kernel(TTArgs A)
{
    __shared__ __align__(16) float hs[TT_H];
    const int l = threadIdx.x;
    const float *W = A.weights;
    TTLane L;
#pragma unroll
    for (int i = 0; i < TT_H; i += 4) {
        const float4 va = *(const float4 *)(W + TT_W2 + l * TT_H + i);
        const float4 vb = *(const float4 *)(W + TT_W2 + (l + 64) * TT_H + i);
        L.w2a[i] = va.x; L.w2a[i + 1] = va.y; L.w2a[i + 2] = va.z; L.w2a[i + 3] = va.w;
        L.w2b[i] = vb.x; L.w2b[i + 1] = vb.y; L.w2b[i + 2] = vb.z; L.w2b[i + 3] = vb.w;
    }
#pragma unroll
    for (int k = 0; k < TT_IN; ++k) {
        L.w1a[k] = W[TT_W1 + l * TT_IN + k];
        L.w1b[k] = W[TT_W1 + (l + 64) * TT_IN + k];
    }
    L.b1a = W[TT_B1 + l]; L.b1b = W[TT_B1 + l + 64];
    L.b2a = W[TT_B2 + l]; L.b2b = W[TT_B2 + l + 64];
    L.w3a = W[TT_W3 + l]; L.w3b = W[TT_W3 + l + 64];
    L.b3 = W[TT_W3 + TT_H];
    for (int64_t b = blockIdx.x; b < A.B; b += gridDim.x) {
        double st[13], fin[3], g0[12], velo[3];
#pragma unroll
        for (int i = 0; i < 13; ++i) st[i] = A.state[b * 13 + i];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            fin[i] = A.final_point[b * 3 + i];
            velo[i] = A.velo[b * 3 + i];
        }
#pragma unroll
        for (int i = 0; i < 12; ++i) g0[i] = A.gate[b * 12 + i];
        double cen[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) cen[a] = ((g0[a] + g0[3 + a]) + g0[6 + a] + g0[9 + a]) / 4.0;
        const double dx = cen[0] - st[0], dy = cen[1] - st[1], dz = cen[2] - st[2];
        double t1 = sqrt(dx * dx + dy * dy + dz * dz) / 3;
        int it = 0;
        for (;;) {                   // one evaluation site: t2 at t1, stop, else halve toward t2
            const double t2 = tt_time_at(L, hs, g0, st, fin, velo, A.w, t1);
            if (!(fabs(t2 - t1) > TT_TOL) || it == TT_MAXIT) break;
            t1 = t1 + (t2 - t1) / 2;
            ++it;
        }
        if (l == 0) {
            A.t_out[b] = t1;
            if (A.iters) A.iters[b] = it;
        }
    }
}

}  // namespace lafse3
