// TEST INFRASTRUCTURE: AddressSanitizer + UndefinedBehaviorSanitizer driver for the device model closed
// forms (csrc/model.hpp through model_host.cpp), host-only hipcc build (tests/native/Makefile target
// model_sanitize), run by tests/test_sanitizers.py.  Seeded pseudo-random states / controls / costates /
// attitudes over the ranges the solver visits; any sanitizer report aborts with a non-zero exit.
#include "model_host.cpp"

#include <cmath>
#include <cstdio>
#include <vector>

static double rnd(unsigned long long &s, double lo, double hi)
{
    s = s * 6364136223846793005ULL + 1442695040888963407ULL;
    return lo + (hi - lo) * (double)(s >> 11) * (1.0 / 9007199254740992.0);
}

int main()
{
    const int n = 257;
    unsigned long long s = 2025;
    std::vector<double> x(n * NX), u(n * NU), lam(n * NX), goal(n * 3), ptra(n * 3), qtra(n * 4), wk(n);
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < NX; ++j) x[i * NX + j] = rnd(s, -5, 5);
        double qn = 0;
        for (int j = 6; j < 10; ++j) qn += x[i * NX + j] * x[i * NX + j];
        for (int j = 6; j < 10; ++j) x[i * NX + j] /= std::sqrt(qn);
        for (int j = 0; j < NU; ++j) u[i * NU + j] = rnd(s, 0, 2.44);
        for (int j = 0; j < NX; ++j) lam[i * NX + j] = rnd(s, -1e3, 1e3);
        for (int j = 0; j < 3; ++j) goal[i * 3 + j] = rnd(s, -10, 10), ptra[i * 3 + j] = rnd(s, -10, 10);
        double q[4], m = 0;
        for (int j = 0; j < 4; ++j) q[j] = rnd(s, -1, 1), m += q[j] * q[j];
        for (int j = 0; j < 4; ++j) qtra[i * 4 + j] = q[j] / std::sqrt(m);
        wk[i] = rnd(s, 0, 60);
    }
    std::vector<double> f(n * NX), A(n * NX * NX), B(n * NX * NU), At(n * NX * NX), Bt(n * NU * NX),
        Hl(n * NX * NX), qu(n * 4), path(n), tra(n), grad(n * NX), hess(n * NX * NX);
    int rc = model_host_eval(n, x.data(), u.data(), lam.data(), f.data(), A.data(), B.data(), At.data(), Bt.data(),
                             Hl.data(), qu.data());
    rc |= model_host_cost(n, x.data(), goal.data(), ptra.data(), qtra.data(), wk.data(), path.data(), tra.data(),
                          grad.data(), hess.data());
    int bad = rc != 0;
    for (double v : A) bad |= !std::isfinite(v);
    for (double v : hess) bad |= !std::isfinite(v);
    std::printf("model_sanitize %s (n=%d)\n", bad ? "FAILED" : "ok", n);
    return bad;
}
