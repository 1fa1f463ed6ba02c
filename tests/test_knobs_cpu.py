"""The build / runtime environment knobs that survived the round-6 cleanup
(README "Environment knobs"): each is read where documented and does what
it says.  Subprocesses, since every knob is read at import time."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _py(code, **env):
    e = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("GPU_MAX_HW_QUEUES", "KFB_HW_QUEUES", "KFB_HIP_LIB", "KFB_NO_AUTOBUILD",
              "KFB_OFFLOAD_ARCH"):
        e.pop(k, None)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True,
                       timeout=300)
    return r


def test_hw_queues_default_and_override():
    code = "import kf_benchmarks_amd, os; print(os.environ['GPU_MAX_HW_QUEUES'])"
    assert _py(code).stdout.strip() == "8"
    assert _py(code, KFB_HW_QUEUES="4").stdout.strip() == "4"
    assert _py(code, KFB_HW_QUEUES="99").stdout.strip() == "32"  # clamped
    # an explicit non-default GPU_MAX_HW_QUEUES is the user's choice
    assert _py(code, GPU_MAX_HW_QUEUES="6").stdout.strip() == "6"


def test_hip_lib_override_and_no_autobuild(tmp_path):
    from kf_benchmarks_amd import build
    code = ("from kf_benchmarks_amd.ops import _native as N; N.load(); "
            "print(N.loaded_path())")
    r = _py(code, KFB_HIP_LIB=build.HIP_LIB)
    assert r.returncode == 0 and r.stdout.strip() == build.HIP_LIB, r.stderr[-2000:]
    missing = str(tmp_path / "nope.so")
    r = _py(code, KFB_HIP_LIB=missing, KFB_NO_AUTOBUILD="1")
    assert r.returncode != 0 and "native kernel library missing" in r.stderr


def test_offload_arch_reaches_hipcc_flags():
    code = "from kf_benchmarks_amd import build; print(build.ARCH, build.HIP_FLAGS)"
    assert "gfx950" in _py(code).stdout
    out = _py(code, KFB_OFFLOAD_ARCH="gfx942").stdout
    assert out.startswith("gfx942") and "--offload-arch=gfx942" in out
