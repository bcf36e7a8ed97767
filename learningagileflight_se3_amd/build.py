"""Build the in-tree HIP library liblafse3.so for gfx950 (and, when asked, the CPU oracle).

    python -m learningagileflight_se3_amd.build

hipcc cross-compiles without a GPU; the .so lands next to this file so it travels with the repo
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "liblafse3.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -amdgpu-disable-unclustered-high-rp-reschedule: the scheduler's high-register-pressure re-scheduling stage
# otherwise reorders the latency-bound sweeps of linear_solve (at the 256-VGPR cap): ipm_kernel 533.4 -> 530.0 ms
# (tools/gpu_variants.sh, two calls, identical iteration counts)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
         "-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule=1",
         "-mllvm", "-amdgpu-mfma-vgpr-form",   # MFMA C/D in VGPRs: no accvgpr copies around the f64 MFMAs (+1.7 %)
         "-mllvm", "-amdgpu-use-amdgpu-trackers",   # the scheduler's AMDGPU register-pressure trackers (+0.9 %, round 5)
         "-mllvm", "-amdgpu-max-memory-clause=31",   # longer load clauses (default 15): +0.2 %, 5 of 5 pairs
         "-I" + os.path.join(REPO, "include")]


def source_hash() -> str:
    """sha256 (16 hex) of what liblafse3.so is built from: csrc/*, include/lafse3.h and the build flags.
    tools/make_pmc_current.py stamps committed PMC profiles with it; bench.py uses a profile's traffic only
    when the stamp equals the tree's (a profile of other kernel sources is stale)."""
    import hashlib
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(CSRC, "*"))) + [os.path.join(REPO, "include", "lafse3.h")]:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS[:-1]).encode())   # the -I path differs between machines
    return h.hexdigest()[:16]


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


OUT_TIMERS = os.path.join(HERE, "liblafse3_timers.so")


def build(force: bool = False, verbose: bool = False, timers: bool = False) -> str:
    """liblafse3.so, or with timers=True the diagnostic liblafse3_timers.so (same ABI, s_memtime phase
    timers compiled in; tools/gpu_timers.py loads it through LAFSE3_LIB)."""
    out = OUT_TIMERS if timers else OUT
    deps = glob.glob(os.path.join(CSRC, "*")) + [os.path.join(REPO, "include", "lafse3.h")]
    if force or _stale(out, deps):
        extra = ["-DLAFSE3_PHASE_TIMERS"] if timers else []
        cmd = [HIPCC] + FLAGS + extra + ["-o", out + ".tmp", os.path.join(CSRC, "api.hip")]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        os.replace(out + ".tmp", out)
    return out


def build_oracle() -> str:
    """TEST INFRASTRUCTURE: compile oracle/ (gcc) for the parity checker and cpu_baseline."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
    return os.path.join(REPO, "oracle", "liblafse3_oracle.so")


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, timers="--timers" in sys.argv))
