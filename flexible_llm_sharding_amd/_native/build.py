"""Build the native libraries in-tree (no torch headers, no JIT cache).

* ``libfls_kernels.so`` — every ``csrc/kernels/*.hip`` compiled by
  ``hipcc --offload-arch=gfx950`` (CDNA4 only) and linked into one library;
* ``libfls_runtime.so`` — ``csrc/runtime/*.cpp`` host runtime (g++ against
  libamdhip64).

Objects are rebuilt only when a source or header is newer.  Usage::

    python -m flexible_llm_sharding_amd._native.build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(HERE, "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("FLS_OFFLOAD_ARCH", "gfx950")   # knobs.py (not imported: the build runs standalone)

KERNELS_SO = os.path.join(HERE, "libfls_kernels.so")
RUNTIME_SO = os.path.join(HERE, "libfls_runtime.so")
COMM_SO = os.path.join(HERE, "libfls_comm.so")


def _hipcc() -> str:
    p = os.path.join(ROCM, "bin", "hipcc")
    return p if os.path.exists(p) else (shutil.which("hipcc") or "hipcc")


def _headers():
    return glob.glob(os.path.join(CSRC, "include", "*.h")) + glob.glob(os.path.join(CSRC, "kernels", "*.cuh")) \
        + glob.glob(os.path.join(CSRC, "kernels", "*.h"))


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    if verbose and r.stdout.strip():
        print(r.stdout)


def build_kernels(force=False, jobs=8, verbose=False, extra_flags=(), variant: str = ""):
    """``variant`` (A/B builds): objects under obj/<variant>/ and the library
    ``variants/libfls_kernels_<variant>.so``, compiled with ``extra_flags`` (e.g. -DV11_SCHED=2)."""
    obj_dir = os.path.join(OBJ, variant) if variant else OBJ
    out_so = os.path.join(HERE, "variants", f"libfls_kernels_{variant}.so") if variant else KERNELS_SO
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(os.path.dirname(out_so), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = _headers()
    inc = ["-I", os.path.join(CSRC, "include"), "-I", os.path.join(CSRC, "kernels")]
    flags = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
             "-munsafe-fp-atomics", "-Wno-unused-result"] + list(extra_flags)
    objs, cmds = [], []
    for s in srcs:
        o = os.path.join(obj_dir, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(o, [s] + hdrs):
            cmds.append([_hipcc()] + flags + inc + ["-c", s, "-o", o])
    if cmds:
        with ThreadPoolExecutor(max(1, jobs)) as ex:
            list(ex.map(lambda c: _run(c, verbose), cmds))
    if force or cmds or _stale(out_so, objs):
        _run([_hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", out_so] + objs, verbose)
    return out_so


def build_runtime(force=False, verbose=False, sanitize=False):
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    deps = srcs + _headers()
    out = RUNTIME_SO if not sanitize else os.path.join(HERE, "libfls_runtime_asan.so")
    if not (force or _stale(out, deps)):
        return out
    cxx = shutil.which("g++") or "g++"
    cmd = [cxx, "-O2", "-g", "-fPIC", "-shared", "-std=c++17", "-D__HIP_PLATFORM_AMD__",
           "-I", os.path.join(CSRC, "include"), "-I", os.path.join(ROCM, "include")]
    if sanitize:
        cmd += ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
    cmd += srcs + ["-L", os.path.join(ROCM, "lib"), "-Wl,-rpath," + os.path.join(ROCM, "lib"),
                   "-lamdhip64", "-lpthread", "-o", out]
    _run(cmd, verbose)
    return out


def build_comm(force=False, verbose=False):
    """libfls_comm.so: the native RCCL communicator (csrc/comm), host code linked to librccl."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp")))
    if not (force or _stale(COMM_SO, srcs + _headers())):
        return COMM_SO
    cxx = shutil.which("g++") or "g++"
    cmd = [cxx, "-O2", "-g", "-fPIC", "-shared", "-std=c++17", "-D__HIP_PLATFORM_AMD__",
           "-I", os.path.join(CSRC, "include"), "-I", os.path.join(ROCM, "include")]
    cmd += srcs + ["-L", os.path.join(ROCM, "lib"), "-Wl,-rpath," + os.path.join(ROCM, "lib"),
                   "-lrccl", "-lamdhip64", "-o", COMM_SO]
    _run(cmd, verbose)
    return COMM_SO


def build_all(force=False, jobs=8, verbose=False):
    rt = build_runtime(force=force, verbose=verbose)
    k = build_kernels(force=force, jobs=jobs, verbose=verbose)
    c = build_comm(force=force, verbose=verbose)
    return rt, k, c


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--variant", default="", help="A/B build: name of a kernel-library variant")
    ap.add_argument("--define", action="append", default=[], help="-D flags of the variant (NAME=VALUE)")
    a = ap.parse_args(argv)
    if a.variant:
        print("built", build_kernels(a.force, a.jobs, a.verbose, ["-D" + d for d in a.define], a.variant))
        return 0
    for p in build_all(a.force, a.jobs, a.verbose):
        print("built", p)


if __name__ == "__main__":
    sys.exit(main())
