"""CPU checks of the C-ABI library: it loads, exports every entry point include/lafse3.h declares,
and its parameter struct / defaults match the reference constants (no device calls)."""
import ctypes
import os
import re

import pytest

from learningagileflight_se3_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "lafse3.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(lafse3_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("liblafse3.so not built: run python -c 'import __graft_entry__ as g; g.build()'")
    return _lib.load()


def test_header_symbols_exported(lib):
    names = _declared()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), f"{n} declared in lafse3.h but not exported"
        assert n in _lib.SIGNATURES, f"{n} has no ctypes signature in _lib.SIGNATURES"


def test_version_names_gfx950(lib):
    assert b"gfx950" in lib.lafse3_version()


def test_params_struct_matches_header_and_reference(lib):
    p = _lib.default_params()
    # sizes: 24 doubles, then the solver block (int32 padding rules identical on both sides)
    assert ctypes.sizeof(_lib.Params) == ctypes.sizeof(p)
    # reference constants: quad_policy.py:37-51, quad_model.py:37, quad_OC.py:145
    assert (p.mass, p.Jx, p.Jy, p.Jz, p.arm_l, p.c_tau, p.grav, p.dt) == (0.5, 0.0023, 0.0023, 0.004, 0.35,
                                                                           0.0245, 9.78, 0.1)
    assert (p.wrt, p.wqt, p.wthrust, p.wrf, p.wvf, p.wqf, p.wwf) == (5, 80, 0.1, 5, 5, 0, 3)
    assert p.horizon == 50 and p.u_lb == 0.0 and abs(p.u_ub - 2.44) < 1e-15
    assert abs(p.w_ub - 3.141592653589793 / 2) < 1e-15 and p.tol == 1e-8
    assert p.costate_option == 0          # IPOPT lam_g, the reference's default (quad_OC.py:104)
    assert p.grad_mode == 0               # FD, the reference's sol_gradient (quad_policy.py:94-112)


def test_workspace_size_positive(lib):
    assert lib.lafse3_workspace_bytes_per_instance() > 0


def test_engine_rejects_mismatched_batch():
    """Every per-sample argument must have ini_state's batch (the kernels read row b < B of each); only u_last
    broadcasts from one row (out-of-bounds device reads otherwise)."""
    import torch
    from learningagileflight_se3_amd.engine import _same_batch
    B = 4
    goal = torch.zeros(B, 3)
    ul1 = torch.ones(1, 4)
    g, ul = _same_batch(B, goal=goal, u_last=ul1)
    assert ul.shape == (B, 4) and g is goal
    with pytest.raises(ValueError, match="gate12"):
        _same_batch(B, goal=goal, gate12=torch.zeros(1, 12))
    with pytest.raises(ValueError, match="dnn_out"):
        _same_batch(B, dnn_out=torch.zeros(3, 7))
    with pytest.raises(ValueError, match="u_last"):
        _same_batch(B, u_last=torch.zeros(2, 4))


def test_stream_create_rejects_null_arguments(lib):
    """lafse3_stream_create / _destroy validate their pointers before any HIP call (LAFSE3_EINVAL, message set)."""
    assert lib.lafse3_stream_create(0, None) == -1
    assert b"null stream" in lib.lafse3_last_error()
    assert lib.lafse3_stream_destroy(None) == -1
