"""CPU unit tests of the DEVICE model closed forms (csrc/model.hpp compiled for the host with hipcc)
against the oracle's dense derivatives (which are pinned to the reference's sympy expressions by
tests/test_oracle_golden.py).  Catches sign/index errors in A^T lam, B^T lam, Hessian-vector products."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "native", "model_host.cpp")
LIB = os.path.join(HERE, "native", "libmodel_host.so")


@pytest.fixture(scope="module")
def host():
    deps = [SRC, os.path.join(REPO, "learningagileflight_se3_amd", "csrc", "model.hpp")]
    if not os.path.exists(LIB) or any(os.path.getmtime(d) > os.path.getmtime(LIB) for d in deps):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O2", "-fPIC", "-shared", "-std=c++17",
                               "-I" + os.path.join(REPO, "include"),
                               "-I" + os.path.join(REPO, "learningagileflight_se3_amd", "csrc"),
                               "-o", LIB, SRC])
    L = ctypes.CDLL(LIB)
    pd = ctypes.POINTER(ctypes.c_double)
    L.model_host_eval.argtypes = [ctypes.c_int] + [pd] * 10
    L.model_host_cost.argtypes = [ctypes.c_int] + [pd] * 9
    return L


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def test_device_jacobians_and_transposes(host, golden):
    g = golden("model")
    n = g["x"].shape[0]
    x, u, lam = [np.ascontiguousarray(g[k]) for k in ("x", "u", "lam")]
    f = np.zeros((n, 13)); A = np.zeros((n, 13, 13)); B = np.zeros((n, 13, 4))
    At = np.zeros((n, 13, 13)); Bt = np.zeros((n, 4, 13)); Hl = np.zeros((n, 13, 13)); qu = np.zeros((n, 4))
    host.model_host_eval(n, _p(x), _p(u), _p(lam), _p(f), _p(A), _p(B), _p(At), _p(Bt), _p(Hl), _p(qu))
    rel = lambda a, b: np.max(np.abs(a - b) / (1 + np.abs(b)))
    assert rel(f, g["f"]) < 1e-13
    assert rel(A, g["A"]) < 1e-13                       # A v
    assert rel(At, np.swapaxes(g["A"], 1, 2)) < 1e-13   # A^T l
    assert rel(B, g["B"]) < 1e-13
    assert rel(Bt, np.swapaxes(g["B"], 1, 2)) < 1e-13
    # lambda-Hessian of f_d: x-x block and q-u coupling (same for every rotor)
    assert rel(Hl, g["Hxx"]) < 1e-13
    assert rel(np.repeat(qu[:, :, None], 4, axis=2), g["Hxu"][:, 6:10, :]) < 1e-13
    assert np.max(np.abs(g["Hxu"][:, [0, 1, 2, 3, 4, 5, 10, 11, 12], :])) == 0.0


def test_device_cost_derivatives(host, golden):
    g = golden("costs")
    n = g["x"].shape[0]
    x = np.ascontiguousarray(g["x"]); goal = np.ascontiguousarray(g["goal"]); ptra = np.ascontiguousarray(g["ptra"])
    qtra = np.ascontiguousarray(g["qtra"]); wk = np.ascontiguousarray(g["wk"])
    path = np.zeros(n); tra = np.zeros(n); grad = np.zeros((n, 13)); hess = np.zeros((n, 13, 13))
    host.model_host_cost(n, _p(x), _p(goal), _p(ptra), _p(qtra), _p(wk), _p(path), _p(tra), _p(grad), _p(hess))
    rel = lambda a, b: np.max(np.abs(a - b) / (1 + np.abs(b)))
    assert rel(path, g["path"]) < 1e-13
    assert rel(tra, g["tra"]) < 1e-11
    assert rel(grad, g["grad"]) < 1e-11
    assert rel(hess, g["hess"]) < 1e-11
