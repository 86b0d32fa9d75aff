"""In-tree native build (no JIT cache, no hipify, no setuptools CUDAExtension).

Compiles every ``csrc/**/*.hip`` with ``hipcc --offload-arch=gfx950`` (device
kernels + their host launchers, no torch headers -> seconds per file) and every
``csrc/**/*.cpp`` (torch/pybind11 bindings, C++ runtime: communicator, reducer,
engine) with hipcc as host C++, then links ONE shared object
``cs744_pytorch_distributed_tutorial_amd/_C.so`` against the HIP/RCCL/torch
libraries that ship inside the installed torch wheel (so the process has exactly
one HIP runtime and one RCCL, SURVEY.md §5.8 "Library pitfall").

Incremental: an object is rebuilt when its source or any header under
``csrc/`` is newer. Usage: ``python -m cs744_pytorch_distributed_tutorial_amd._build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
import time

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "obj")
OUT = os.path.join(PKG_DIR, "_C.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, os.path.join(tdir, "lib")


def _sources():
    tests = os.path.join(CSRC, "tests") + os.sep
    hip = sorted(f for f in glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True) if not f.startswith(tests))
    cpp = sorted(f for f in glob.glob(os.path.join(CSRC, "**", "*.cpp"), recursive=True) if not f.startswith(tests))
    return hip, cpp


def _deps_mtime(obj: str) -> float:
    """Newest in-tree header the object was compiled against (from the -MD depfile), or
    +inf when the depfile is missing (forces a rebuild). Out-of-tree headers (torch, ROCm)
    are skipped: they only change with the image."""
    dep = obj + ".d"
    if not os.path.exists(dep):
        return float("inf")
    with open(dep) as f:
        text = f.read().replace("\\\n", " ")
    newest = 0.0
    for tok in text.split(":", 1)[-1].split():
        if tok.startswith(CSRC):
            if not os.path.exists(tok):
                return float("inf")
            newest = max(newest, os.path.getmtime(tok))
    return newest


def _obj_path(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(BUILD, rel + ".o")


def _common_flags():
    return ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC}", "-D__HIP_PLATFORM_AMD__", "-Wno-unused-result",
            "-Wno-unused-command-line-argument"]


def _compile_cmd(src: str, obj: str):
    if src.endswith(".hip"):
        return [HIPCC, f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *_common_flags(), "-MD", "-MF", obj + ".d",
                "-c", src, "-o", obj]
    _, tinc, _ = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    incs = [f"-I{p}" for p in tinc] + [f"-I{py_inc}", f"-I{ROCM}/include"]
    return [HIPCC, *_common_flags(), *incs, "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
            "-D_GLIBCXX_USE_CXX11_ABI=1", "-DUSE_ROCM=1", "-MD", "-MF", obj + ".d", "-x", "c++", "-c", src,
            "-o", obj]


def _link_cmd(objs, out=OUT):
    _, _, tlib = _torch_paths()
    return [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fgpu-rdc" if False else "-fPIC", "-o", out, *objs,
            f"-L{tlib}", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lc10", "-lc10_hip", "-ltorch_python",
            "-l:libamdhip64.so", "-l:librccl.so", f"-Wl,-rpath,{tlib}", "-Wl,--no-as-needed"]


def build(jobs: int = 0, force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hip, cpp = _sources()
    todo = []
    objs = []
    for s in hip + cpp:
        o = _obj_path(s)
        objs.append(o)
        if force or not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), _deps_mtime(o)):
            todo.append((s, o))
    jobs = jobs or min(8, os.cpu_count() or 4)
    t0 = time.time()
    if todo:
        def run(so):
            s, o = so
            cmd = _compile_cmd(s, o)
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"compile failed: {os.path.relpath(s, ROOT)}\n{r.stdout}\n{r.stderr}")
            return s
        with cf.ThreadPoolExecutor(jobs) as ex:
            for s in ex.map(run, todo):
                print(f"[build] compiled {os.path.relpath(s, ROOT)}", flush=True)
    if todo or not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs):
        # link to a temporary name and rename: a reader (an import, a tree snapshot) never sees a
        # half-written library
        tmp = OUT + f".tmp{os.getpid()}"
        cmd = _link_cmd(objs, tmp)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            if os.path.exists(tmp):
                os.remove(tmp)
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        _check_stubs(tmp)
        os.replace(tmp, OUT)
        print(f"[build] linked {os.path.relpath(OUT, ROOT)} ({len(objs)} objects, {time.time() - t0:.1f}s)",
              flush=True)
    return OUT


def _check_stubs(so: str) -> None:
    """Fail the build if a kernel's host stub is left undefined (hipcc can drop implicitly
    instantiated template-kernel stubs; the .so would then fail at import on the GPU box)."""
    nm = os.path.join(ROCM, "lib", "llvm", "bin", "llvm-nm")
    if not os.path.exists(nm):
        return
    r = subprocess.run([nm, "--undefined-only", "-C", so], capture_output=True, text=True)
    bad = [l.strip() for l in r.stdout.splitlines() if "__device_stub__" in l]
    if bad:
        os.remove(so)
        raise RuntimeError("undefined kernel stubs (add explicit instantiations):\n" + "\n".join(bad[:10]))


ASAN_OUT = os.path.join(PKG_DIR, "bin", "asan_runtime_test")
# host code only: device code is never sanitized (each -fsanitize right after -Xarch_host)
ASAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer", "-O1", "-gline-tables-only"]


def build_asan(jobs: int = 0, verbose: bool = False) -> str:
    """Standalone AddressSanitizer build of the C++ runtime (runtime/*.cpp) and
    csrc/tests/asan_runtime_test.cpp, linked against the product build's kernel
    objects (device code is never sanitized, so the kernels and their launchers are the
    ``build()`` objects as they are — a separate ASan object tree for the runtime only, and a
    program a fraction of the size of an all-sanitized one). The product _C.so is untouched."""
    build(jobs)  # the kernel objects (incremental)
    obj_dir = os.path.join(ROOT, "build", "asan")
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(os.path.dirname(ASAN_OUT), exist_ok=True)
    hip_objs = [_obj_path(f) for f in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))]
    cpp = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))) + [os.path.join(CSRC, "tests", "asan_runtime_test.cpp")]
    _, tinc, tlib = _torch_paths()
    incs = [f"-I{p}" for p in tinc] + [f"-I{sysconfig.get_paths()['include']}", f"-I{ROCM}/include"]
    todo, objs = [], list(hip_objs)
    for src in cpp:
        o = os.path.join(obj_dir, os.path.relpath(src, CSRC).replace(os.sep, "__") + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(src), _deps_mtime(o)):
            cmd = [HIPCC, *_common_flags(), *ASAN_FLAGS, *incs, "-D_GLIBCXX_USE_CXX11_ABI=1", "-DUSE_ROCM=1",
                   "-MD", "-MF", o + ".d", "-x", "c++", "-c", src, "-o", o]
            todo.append((src, cmd))

    def run(item):
        src, cmd = item
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"asan compile failed: {os.path.relpath(src, ROOT)}\n{r.stdout}\n{r.stderr}")
        return src
    with cf.ThreadPoolExecutor(jobs or min(8, os.cpu_count() or 4)) as ex:
        for src in ex.map(run, todo):
            print(f"[build:asan] compiled {os.path.relpath(src, ROOT)}", flush=True)
    # One copy of every ROCm runtime library: torch ships them under file names without the
    # soname's version suffix, so a standalone program's NEEDED "libamdhip64.so.7" would resolve
    # to /opt/rocm while libtorch_hip loads torch's copy (two HIP / RCCL / SMI runtimes; ASan
    # then reports the SMI library's static map freed twice at exit). bin/libs/<soname> ->
    # torch's file, searched first through $ORIGIN (same torch install on the GPU box).
    libs = os.path.join(os.path.dirname(ASAN_OUT), "libs")
    os.makedirs(libs, exist_ok=True)
    for f in glob.glob(os.path.join(tlib, "*.so")):
        r = subprocess.run([os.path.join(ROCM, "lib", "llvm", "bin", "llvm-readelf"), "-d", f], capture_output=True,
                           text=True)
        son = [l.split("[")[-1].rstrip("]") for l in r.stdout.splitlines() if "SONAME" in l]
        if son and son[0] != os.path.basename(f):
            link = os.path.join(libs, son[0])
            if os.path.lexists(link):
                os.remove(link)
            os.symlink(f, link)
    cmd = [HIPCC, f"--offload-arch={ARCH}", *ASAN_FLAGS, "-o", ASAN_OUT, *objs, f"-L{tlib}", "-ltorch", "-ltorch_cpu",
           "-ltorch_hip", "-lc10", "-lc10_hip", "-l:libamdhip64.so", "-l:librccl.so", "-Wl,--disable-new-dtags",
           "-Wl,-rpath,$ORIGIN/libs", f"-Wl,-rpath,{tlib}", "-Wl,--no-as-needed"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"asan link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    print(f"[build:asan] linked {os.path.relpath(ASAN_OUT, ROOT)}", flush=True)
    return ASAN_OUT


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("-j", "--jobs", type=int, default=0)
    p.add_argument("--force", action="store_true")
    p.add_argument("-v", "--verbose", action="store_true")
    p.add_argument("--asan", action="store_true", help="also build the host-ASan runtime test program")
    a = p.parse_args(argv)
    build(a.jobs, a.force, a.verbose)
    if a.asan:
        build_asan(a.jobs, a.verbose)
    return 0


if __name__ == "__main__":
    sys.exit(main())
