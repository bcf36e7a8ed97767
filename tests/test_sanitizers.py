"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer runs (CPU only; GPU sanitizers are not
available on the MI355X pool and no GPU code is instrumented here).

tests/native/Makefile builds two drivers with -fsanitize=address,undefined -fno-sanitize-recover=all:
  * oracle_sanitize -- oracle/lafse3_oracle.c (gcc): both gradient modes, u_last, horizon 20, the
    reward / collision scorer, model / cost derivative dumps and the trace/dump debug hooks, on a
    seeded synthetic batch written here;
  * model_sanitize  -- the device model closed forms csrc/model.hpp through tests/native/model_host.cpp
    (hipcc host-only compilation), on seeded random points.
Any sanitizer report makes the driver exit non-zero and prints the report, which fails the test.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")


@pytest.fixture(scope="module")
def san_dir(tmp_path_factory):
    if shutil.which("gcc") is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("gcc / hipcc not available")
    out = str(tmp_path_factory.mktemp("san"))
    subprocess.run(["make", "-s", "-C", NATIVE, "OUT=" + out], check=True, capture_output=True, timeout=600)
    return out


def _run(cmd, timeout):
    # verify_asan_link_order=0: the environment may preload a library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0 and "runtime error" not in r.stderr, r.stdout + r.stderr
    return r.stdout


def test_oracle_under_asan_ubsan(san_dir, tmp_path):
    from learningagileflight_se3_amd import scenario as S
    sb = S.synthetic_batch(2, seed=5)
    B = 2
    buf = np.concatenate([[float(B)], sb["ini"].ravel(), sb["goal"].ravel(), sb["gate12"].ravel(),
                          sb["dnn_out"].astype(np.float64).ravel()]).astype(np.float64)
    f = tmp_path / "in.bin"
    buf.tofile(str(f))
    out = _run([os.path.join(san_dir, "oracle_sanitize"), str(f)], 900)
    assert "oracle_sanitize ok" in out


def test_device_model_host_build_under_asan_ubsan(san_dir):
    out = _run([os.path.join(san_dir, "model_sanitize")], 300)
    assert "model_sanitize ok" in out
