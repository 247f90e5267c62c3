"""Build the native libraries in-tree (no JIT cache: the ``.so`` files travel with the repo).

* ``rocket_amd/_lib/librocket_kernels.so`` — every ``native/kernels/*.hip``
  compiled for ``gfx950`` (CDNA4) only;
* ``rocket_amd/_lib/librocket_runtime.so`` — the C++ runtime in
  ``native/runtime/*.cpp`` (RCCL communicator + gradient reducer, pinned
  batch gatherer), linked against RCCL and the HIP runtime.

Objects are rebuilt only when a source or header is newer than its object;
compilation runs in parallel.  ``python -m rocket_amd.native.build [--force]``.
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
LIBDIR = os.path.join(PKG, "_lib")
OBJDIR = os.path.join(LIBDIR, "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("ROCKET_OFFLOAD_ARCH", "gfx950")

KERNELS_SO = os.path.join(LIBDIR, "librocket_kernels.so")
RUNTIME_SO = os.path.join(LIBDIR, "librocket_runtime.so")


def _hipcc() -> str:
    for c in (os.path.join(ROCM, "bin", "hipcc"), shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build rocket_amd native kernels)")


def _newest(paths) -> float:
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def _compile(cmd, out) -> str:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return out


def _included_sources(src) -> list:
    """Sources a translation unit textually includes (e.g. lenet_conv_h.hip: #include "lenet_conv.hip")."""
    d = os.path.dirname(src)
    with open(src) as f:
        names = re.findall(r'^\s*#\s*include\s+"([^"]+\.(?:hip|cpp))"', f.read(), flags=re.M)
    return [os.path.join(d, n) for n in names if os.path.exists(os.path.join(d, n))]


def _build_lib(sources, headers, target, extra_compile, extra_link, force, jobs, language_hip=True) -> bool:
    os.makedirs(OBJDIR, exist_ok=True)
    hipcc = _hipcc()
    hdr_time = _newest(headers)
    objs, todo = [], []
    for src in sources:
        obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
        objs.append(obj)
        src_time = _newest([src] + _included_sources(src))
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(src_time, hdr_time):
            flags = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", f"-I{os.path.dirname(src)}"]
            if language_hip:
                flags += [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
            else:
                flags += ["-x", "c++", "-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include"]
            todo.append(([hipcc] + flags + extra_compile + ["-c", src, "-o", obj], obj))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda a: _compile(*a), todo))
    if force or todo or not os.path.exists(target) or os.path.getmtime(target) < _newest(objs):
        cmd = [hipcc, "-shared", "-fPIC", "-o", target] + objs + extra_link
        if language_hip:
            cmd.insert(1, f"--offload-arch={ARCH}")
        _compile(cmd, target)
        return True
    return False


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> dict:
    jobs = jobs or min(8, os.cpu_count() or 4)
    kdir = os.path.join(HERE, "kernels")
    rdir = os.path.join(HERE, "runtime")
    built = {}
    ksrc = sorted(glob.glob(os.path.join(kdir, "*.hip")))
    khdr = glob.glob(os.path.join(kdir, "*.h"))
    if ksrc:
        built["kernels"] = _build_lib(ksrc, khdr, KERNELS_SO, [], [], force, jobs)
    rsrc = sorted(glob.glob(os.path.join(rdir, "*.cpp")))
    rhdr = glob.glob(os.path.join(rdir, "*.h"))
    if rsrc:
        built["runtime"] = _build_lib(
            rsrc, rhdr, RUNTIME_SO, [], [f"-L{ROCM}/lib", "-lrccl", "-lamdhip64", "-lpthread", f"-Wl,-rpath,{ROCM}/lib"],
            force, jobs, language_hip=False,
        )
    if verbose:
        print(f"[rocket_amd.native] built={built} -> {LIBDIR}")
    return built


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args()
    try:
        build(force=a.force, jobs=a.j)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
