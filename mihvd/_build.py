"""In-tree native build for mihvd.

Two shared objects are produced under ``mihvd/_native/``:

* ``_mihvd_runtime*.so`` — the C++ host runtime (``csrc/runtime``), a pybind11 module built with
  g++. It needs no GPU and is used by the CPU tests.
* ``libmihvd_kernels.so`` — the hand-written CDNA4 HIP kernels (``csrc/kernels``), compiled with
  ``hipcc --offload-arch=gfx950`` directly (no hipify, no torch JIT cache) and registered as
  ``torch.ops.mihvd.*`` through ``TORCH_LIBRARY``. It is loaded with ``torch.ops.load_library``.

Both builds are incremental (mtime based) and run in-tree so the ``.so`` files travel with the
repository snapshot to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(ROOT, "mihvd", "_native")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("MIHVD_OFFLOAD_ARCH", "gfx950")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


RUNTIME_SO = os.path.join(OUT, "_mihvd_runtime" + _ext_suffix())
KERNELS_SO = os.path.join(OUT, "libmihvd_kernels.so")


def _newer(target: str, deps) -> bool:
    """True if target is missing or older than any dependency."""
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, cwd=None):
    proc = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("build command failed:\n  %s\n%s" % (" ".join(cmd), proc.stdout))
    return proc.stdout


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cc")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.h")))
    if not force and not _newer(RUNTIME_SO, srcs + hdrs + [__file__]):
        return RUNTIME_SO
    import pybind11

    os.makedirs(OUT, exist_ok=True)
    cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
    inc = [
        "-I" + pybind11.get_include(),
        "-I" + sysconfig.get_paths()["include"],
        "-I" + os.path.join(CSRC, "runtime"),
    ]
    tmp = RUNTIME_SO + ".tmp%d" % os.getpid()
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-pthread", *inc,
           *srcs, "-o", tmp]
    out = _run(cmd)
    os.replace(tmp, RUNTIME_SO)
    if verbose and out:
        print(out)
    return RUNTIME_SO


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (set HIPCC)")


# MFMA kernel sources compiled a second time with fp16 operands (-DMIHVD_F16).
F16_SOURCES = ("conv_fwd.hip", "conv_bwd.hip", "fc.hip")


def build_kernels(force: bool = False, verbose: bool = False, jobs: int | None = None) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")) + glob.glob(os.path.join(CSRC, "kernels", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")) + glob.glob(os.path.join(CSRC, "kernels", "*.cuh")))
    if not srcs:
        raise RuntimeError("no kernel sources under csrc/kernels")
    # extra defines of a study build go into a flags stamp the rebuild check compares, so a stamped
    # (instrumented) build is never silently kept by a later normal import, nor skipped by one
    defines = ["-DMIHVD_F32_STAMPS=1"] if os.environ.get("MIHVD_F32_STAMPS") == "1" else []
    os.makedirs(BUILD, exist_ok=True)
    stamp = os.path.join(BUILD, "kernel_flags.txt")
    old = open(stamp).read() if os.path.exists(stamp) else ""
    if old != " ".join(defines):
        force = True
    if not force and not _newer(KERNELS_SO, srcs + hdrs + [__file__]):
        return KERNELS_SO
    tdir, tinc, tlib, abi = _torch_paths()
    hipcc = _hipcc()
    os.makedirs(OUT, exist_ok=True)
    os.makedirs(BUILD, exist_ok=True)
    common = [
        "-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=%d" % abi, "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-Wno-unused-result", "-Wno-deprecated-declarations", "-Wno-unused-command-line-argument",
        "-I" + os.path.join(CSRC, "kernels"), *["-I" + p for p in tinc],
    ]
    if os.environ.get("MIHVD_SAVE_TEMPS"):
        common += ["-save-temps=obj"]
    common += defines  # study build: in-kernel phase stamps (scripts/stamps_f32.py)

    def compile_one(src):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        if force or _newer(obj, [src] + hdrs + [__file__]):
            cmd = [hipcc, *common, "-c", src, "-o", obj]
            if src.endswith(".cpp"):
                cmd = [hipcc, "-x", "hip", *common, "-c", src, "-o", obj]
            _run(cmd, cwd=BUILD)
        return obj

    def compile_f16(src):
        # the fp16-operand build of the MFMA kernels (common.h: namespace mihvd::f16, v_mfma_*_f16)
        obj = os.path.join(BUILD, os.path.basename(src) + ".f16.o")
        if force or _newer(obj, [src] + hdrs + [__file__]):
            _run([hipcc, *common, "-DMIHVD_F16=1", "-c", src, "-o", obj], cwd=BUILD)
        return obj

    jobs = jobs or min(8, os.cpu_count() or 4)
    f16_srcs = [s for s in srcs if os.path.basename(s) in F16_SOURCES]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, srcs)) + list(ex.map(compile_f16, f16_srcs))
    tmp = KERNELS_SO + ".tmp%d" % os.getpid()
    link = [hipcc, "-shared", "-fPIC", "--offload-arch=" + ARCH, *objs, "-L" + tlib, "-ltorch", "-ltorch_cpu",
            "-lc10", "-lc10_hip", "-ltorch_hip", "-Wl,-rpath," + tlib, "-o", tmp]
    _run(link, cwd=BUILD)
    os.replace(tmp, KERNELS_SO)
    with open(stamp, "w") as f:
        f.write(" ".join(defines))
    return KERNELS_SO


SANITIZERS = {
    "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread"],
}


def _sanitizer_cxx() -> str:
    # ROCm's clang: its TSan runtime intercepts pthread_cond_clockwait (libstdc++'s
    # condition_variable::wait_for), which GCC 11's libtsan misses — that produces false
    # "double lock" reports on every cv wait.
    for c in (os.environ.get("MIHVD_SANITIZER_CXX"), "/opt/rocm/llvm/bin/clang++", shutil.which("clang++"),
              shutil.which("g++")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("no C++ compiler for the sanitizer self-test")


def build_selftest(kind: str = "asan", force: bool = False) -> str:
    """Build the host-runtime self-test (csrc/runtime/tests/selftest.cc) under a sanitizer
    (SURVEY.md §5.2): ``asan`` = AddressSanitizer + UndefinedBehaviorSanitizer, ``tsan`` =
    ThreadSanitizer. Host code only: GPU sanitizers are not available for gfx950 on this pool."""
    flags = SANITIZERS[kind]
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cc"))) + [os.path.join(CSRC, "runtime", "tests",
                                                                                    "selftest.cc")]
    hdrs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.h")))
    out_dir = os.path.join(BUILD, "selftest_" + kind)
    exe = os.path.join(out_dir, "selftest")
    srcs = [s for s in srcs if not s.endswith("bindings.cc")]  # pybind11 module entry point
    if not force and not _newer(exe, srcs + hdrs + [__file__]):
        return exe
    os.makedirs(out_dir, exist_ok=True)
    cxx = _sanitizer_cxx()
    common = ["-std=c++17", "-O1", "-g", "-pthread", "-I" + os.path.join(CSRC, "runtime"), *flags]

    def compile_one(src):
        obj = os.path.join(out_dir, os.path.basename(src) + ".o")
        _run([cxx, *common, "-c", src, "-o", obj])
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(compile_one, srcs))
    _run([cxx, *flags, "-pthread", *objs, "-o", exe + ".tmp"])
    os.replace(exe + ".tmp", exe)
    return exe


def build_all(force: bool = False, verbose: bool = False):
    r = build_runtime(force=force, verbose=verbose)
    k = build_kernels(force=force, verbose=verbose)
    return r, k


if __name__ == "__main__":
    force = "--force" in sys.argv
    what = [a for a in sys.argv[1:] if not a.startswith("--")] or ["all"]
    if "runtime" in what or "all" in what:
        print(build_runtime(force=force, verbose=True))
    if "kernels" in what or "all" in what:
        print(build_kernels(force=force, verbose=True))
    for kind in ("asan", "tsan"):
        if "selftest-" + kind in what:
            print(build_selftest(kind, force=force))
