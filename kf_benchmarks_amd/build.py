"""Builds the native libraries in-tree.

* ``_lib/libkfb_hip.so``  - every HIP kernel under ``csrc/*.hip`` for gfx950,
  compiled by ``hipcc --offload-arch=gfx950`` (one object per source, in
  parallel, rebuilt only when a source or header is newer than its object).
* ``_lib/libkfb_rt.so``   - host-side C++ runtime (``csrc/runtime/*.cpp``:
  TFRecord reader/CRC32C, checkpoint bundle index, ...), built with g++.

Both are loaded with ctypes by :mod:`kf_benchmarks_amd.ops._native` and
:mod:`kf_benchmarks_amd.runtime`; neither needs the torch C++ headers, which
keeps a full rebuild to seconds.

Usage: ``python -m kf_benchmarks_amd.build [--force] [-j N]``
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "_lib")
OBJDIR = os.path.join(PKG, "_lib", "obj")
HIP_LIB = os.path.join(LIBDIR, "libkfb_hip.so")
RT_LIB = os.path.join(LIBDIR, "libkfb_rt.so")
ARCH = os.environ.get("KFB_OFFLOAD_ARCH", "gfx950")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HIP_FLAGS = ["-O3", "-fPIC", "-std=c++17", "--offload-arch=%s" % ARCH,
             "-Wno-unused-result", "-munsafe-fp-atomics", "-I", CSRC]
CXX = os.environ.get("CXX", "g++")
CXX_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-I", CSRC]


def _newest_header(dirpath):
    hs = glob.glob(os.path.join(dirpath, "*.h")) + glob.glob(os.path.join(dirpath, "**", "*.h"),
                                                            recursive=True)
    return max([os.path.getmtime(h) for h in hs] + [0.0])


def _stale(src, obj, hdr_time):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or hdr_time > t


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: %s\n%s" % (" ".join(cmd), r.stdout))
    return r.stdout


def hip_sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def rt_sources():
    return sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))


def build_hip(force=False, jobs=None, verbose=False):
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = hip_sources()
    hdr = _newest_header(CSRC)
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(OBJDIR, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(s, o, hdr):
            todo.append((s, o))
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_run, [HIPCC] + HIP_FLAGS + ["-c", s, "-o", o]) for s, o in todo]
        for f in futs:
            out = f.result()
            if verbose and out.strip():
                print(out)
    if todo or force or not os.path.exists(HIP_LIB):
        tmp = HIP_LIB + ".tmp"
        _run([HIPCC, "-shared", "-fPIC", "--offload-arch=%s" % ARCH, "-o", tmp] + objs)
        _check_no_missing_stubs(tmp)
        os.replace(tmp, HIP_LIB)
    return HIP_LIB


def _check_no_missing_stubs(lib):
    """A kernel template the host pass silently dropped leaves its launch
    stub undefined: the link succeeds and only dlopen fails (on the GPU box).
    Catch it here instead."""
    nm = shutil.which("nm")
    if nm is None:
        return
    out = subprocess.run([nm, "-u", lib], stdout=subprocess.PIPE, text=True).stdout
    missing = [l.split()[-1] for l in out.splitlines() if "__device_stub__" in l]
    if missing:
        raise RuntimeError("undefined kernel launch stubs in %s: %s" % (lib, missing))


# jpeglib.h for the native image pipeline (csrc/runtime/kfb_images.cpp); the
# library itself is dlopen'ed at run time, so a build without the header just
# leaves the pipeline unavailable (Python's PIL path runs instead)
JPEG_INCLUDE = os.environ.get("KFB_JPEG_INCLUDE", "/opt/conda/include")


def _jpeg_flags():
    if os.path.exists(os.path.join(JPEG_INCLUDE, "jpeglib.h")):
        return ["-DKFB_HAVE_JPEGLIB", "-idirafter", JPEG_INCLUDE]
    return []


def build_rt(force=False):
    srcs = rt_sources()
    if not srcs:
        return None
    os.makedirs(LIBDIR, exist_ok=True)
    hdr = _newest_header(os.path.join(CSRC, "runtime"))
    newest = max([os.path.getmtime(s) for s in srcs] + [hdr])
    if force or not os.path.exists(RT_LIB) or os.path.getmtime(RT_LIB) < newest:
        tmp = RT_LIB + ".tmp"
        _run([CXX] + CXX_FLAGS + _jpeg_flags() + ["-shared", "-o", tmp] + srcs
             + ["-lpthread", "-ldl"])
        os.replace(tmp, RT_LIB)
    return RT_LIB


RUN_BIN = os.path.join(LIBDIR, "kfb-run")


def build_launcher(force=False):
    """``kfb-run``: the multi-process launcher (csrc/launcher/kfb_run.cpp)."""
    src = os.path.join(CSRC, "launcher", "kfb_run.cpp")
    if not os.path.exists(src):
        return None
    os.makedirs(LIBDIR, exist_ok=True)
    if force or not os.path.exists(RUN_BIN) or os.path.getmtime(RUN_BIN) < os.path.getmtime(src):
        tmp = RUN_BIN + ".tmp"
        _run([CXX, "-O2", "-std=c++17", "-Wall", "-o", tmp, src])
        os.replace(tmp, RUN_BIN)
    return RUN_BIN


def build_all(force=False, jobs=None, verbose=False):
    if shutil.which(HIPCC) is None and not os.path.exists(HIPCC):
        raise RuntimeError("hipcc not found at %s" % HIPCC)
    libs = [build_hip(force=force, jobs=jobs, verbose=verbose)]
    for extra in (build_rt(force=force), build_launcher(force=force)):
        if extra:
            libs.append(extra)
    return libs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args(argv)
    for lib in build_all(force=a.force, jobs=a.j, verbose=a.v):
        print("built", lib)


if __name__ == "__main__":
    sys.exit(main())
