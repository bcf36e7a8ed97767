// riccati_tables.hpp — compile-time sparsity tables of the stage QP used by the Riccati sweeps.
//
// Stage variables z = [x~ (17) ; u (4)] with x~ = [r v q w (13) ; u_prev (4)].
// G = [A~ B~] (17 x 21) is stored as 21 column lists of 7 (row, value) pairs; row indices are the
// fixed structure of d f_d / d(x, u) (quad_model.py:86-119 + Euler step quad_OC.py:52):
//   col r_a : (r_a, 1)
//   col v_a : (r_a, dt) (v_a, 1)
//   col q_c : rows v0..v2 (dt T/m dg/dq)  q0..q3 (I + dt/2 Omega(w))
//   col w_c : rows q0..q3 (dt/2 Xi(q))    w0..w2 (I + dt dw_dot/dw)
//   col u~_a: empty (A~ has zero u_prev columns)
//   col u_a : rows v0..v2 (dt/m g(q))     w0..w2 (rotor torque map)   u~_a (1)
// 54 of the 147 slots vary with the stage; the rest are per-instance constants.
// H~ (stage Hessian, 21 x 21 symmetric) has 62 upper-triangle nonzeros (listed below).
#pragma once

namespace lafse3 {

constexpr int GLEN = 7;     // entries per G column list
constexpr int NGV = 54;     // stage-dependent G slots
constexpr int NHV = 62;     // upper-triangle nonzeros of H~
constexpr int NUP = 231;    // upper triangle of a 21 x 21
constexpr int NUP17 = 153;  // upper triangle of a 17 x 17

// stage table layout (doubles per stage)
constexpr int TB_G = 0;
constexpr int TB_H = TB_G + NGV;       // 54
constexpr int TB_h = TB_H + NHV;       // 116
constexpr int TB_c = TB_h + 21;        // 137
// per-row constants read by the MFMA stage's gathers (riccati_mfma.inc): 1, dt, bwx, -bwx, bwy, -bwy, bwz, -bwz
constexpr int TB_K = TB_c + 13;        // 150
constexpr int TB_W = 160;              // padded row width (multiple of 8 doubles)

__host__ __device__ constexpr int g_row(int j, int t)
{
    // row index of entry t of column j (-1: padding)
    return j < 3 ? (t == 0 ? j : -1)
         : j < 6 ? (t == 0 ? j - 3 : (t == 1 ? j : -1))
         : j < 10 ? 3 + t                   // v0..v2, q0..q3
         : j < 13 ? 6 + t                   // q0..q3, w0..w2
         : j < 17 ? -1
         : (t < 3 ? 3 + t : (t < 6 ? 7 + t : 13 + (j - 17)));
}

// column j and list position t of stage-dependent G slot v
__host__ __device__ constexpr int gv_col(int v)
{
    return v < 24 ? 6 + v / 6 : (v < 42 ? 10 + (v - 24) / 6 : 17 + (v - 42) / 3);
}
__host__ __device__ constexpr int gv_pos(int v)
{
    return v < 24 ? ((v % 6) < 3 ? (v % 6) : 3 + ((v % 6) - 3) + (((v % 6) - 3) >= (v / 6) ? 1 : 0))
         : v < 42 ? (((v - 24) % 6) < 4 ? ((v - 24) % 6)
                                          : 4 + (((v - 24) % 6) - 4) + ((((v - 24) % 6) - 4) >= ((v - 24) / 6) ? 1 : 0))
                  : (v - 42) % 3;
}

// H~ upper-triangle nonzero e: (row, col, flag) with flag 1 = x diagonal (+delta_w when k >= 1),
// 2 = u diagonal (+delta_w)
struct HEnt {
    unsigned char i, j, flag;
};

struct HTab {
    HEnt e[NHV];
    signed char idx[21 * 21];   // (i,j) with i <= j -> H entry or -1
};

__host__ __device__ constexpr HTab make_htab()
{
    HTab T{};
    int n = 0;
    for (int a = 0; a < 3; ++a) T.e[n++] = {(unsigned char)a, (unsigned char)a, 1};              // r
    for (int a = 0; a < 3; ++a) T.e[n++] = {(unsigned char)(3 + a), (unsigned char)(3 + a), 1};  // v
    for (int b = 0; b < 4; ++b)                                                                   // q-q
        for (int c = b; c < 4; ++c)
            T.e[n++] = {(unsigned char)(6 + b), (unsigned char)(6 + c), (unsigned char)(b == c ? 1 : 0)};
    for (int b = 0; b < 4; ++b)                                                                   // q-w
        for (int c = 0; c < 3; ++c) T.e[n++] = {(unsigned char)(6 + b), (unsigned char)(10 + c), 0};
    for (int c = 0; c < 3; ++c)                                                                   // w-w
        for (int d = c; d < 3; ++d)
            T.e[n++] = {(unsigned char)(10 + c), (unsigned char)(10 + d), (unsigned char)(c == d ? 1 : 0)};
    for (int b = 0; b < 4; ++b)                                                                   // q-u
        for (int a = 0; a < 4; ++a) T.e[n++] = {(unsigned char)(6 + b), (unsigned char)(17 + a), 0};
    for (int a = 0; a < 4; ++a) T.e[n++] = {(unsigned char)(13 + a), (unsigned char)(13 + a), 0}; // u~-u~
    for (int a = 0; a < 4; ++a) T.e[n++] = {(unsigned char)(13 + a), (unsigned char)(17 + a), 0}; // u~-u
    for (int a = 0; a < 4; ++a) T.e[n++] = {(unsigned char)(17 + a), (unsigned char)(17 + a), 2}; // u-u
    for (int k = 0; k < 21 * 21; ++k) T.idx[k] = -1;
    for (int k = 0; k < NHV; ++k) T.idx[T.e[k].i * 21 + T.e[k].j] = (signed char)k;
    return T;
}

struct UpTab {
    unsigned char i[NUP], j[NUP];
    unsigned char i17[NUP17], j17[NUP17];
};

__host__ __device__ constexpr UpTab make_uptab()
{
    UpTab T{};
    int n = 0;
    for (int i = 0; i < 21; ++i)
        for (int j = i; j < 21; ++j) {
            T.i[n] = (unsigned char)i;
            T.j[n] = (unsigned char)j;
            ++n;
        }
    n = 0;
    for (int i = 0; i < 17; ++i)
        for (int j = i; j < 17; ++j) {
            T.i17[n] = (unsigned char)i;
            T.j17[n] = (unsigned char)j;
            ++n;
        }
    return T;
}

// index of (i,j) in the packed upper triangle of a 17 x 17
__host__ __device__ constexpr int up17(int i, int j)
{
    return i <= j ? i * 17 - i * (i - 1) / 2 + (j - i) : j * 17 - j * (j - 1) / 2 + (i - j);
}

}  // namespace lafse3
