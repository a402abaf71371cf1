"""In-tree build of the native libraries (no JIT cache, no site-packages).

* ``_lib/libtde_hip.so``  — CDNA4 (gfx950) HIP kernels + RCCL communicator,
  built with ``hipcc --offload-arch=gfx950``.
* ``_lib/libtde_host.so`` — host C++ runtime (TCP store / RPC, parameter
  server, TensorBundle checkpoint + crc32c, TF event writer, batch assembler),
  built with ``g++``; has no HIP dependency so the CPU plumbing path uses it too.

Both are plain C-ABI shared objects loaded with ctypes *after* ``import torch``
so the HIP runtime / RCCL that torch already mapped (same SONAMEs) are reused.

Usage: ``python -m tensorflow_distributed_example_amd._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = ROOT / "csrc"
LIBDIR = PKG / "_lib"
OBJDIR = ROOT / "build" / "obj"

HIP_SOURCES = sorted((CSRC / "kernels").glob("*.hip")) + [CSRC / "comm" / "rccl_comm.cpp",
                                                           CSRC / "comm" / "xgmi_allreduce.hip"]
HOST_DIRS = ["host", "io", "ps", "data"]


def _host_sources():
    out = []
    for d in HOST_DIRS:
        out += sorted((CSRC / d).glob("*.cpp"))
    out += [p for p in sorted((CSRC / "comm").glob("*.cpp")) if p.name != "rccl_comm.cpp"]
    return out


def _rocm():
    return os.environ.get("ROCM_PATH", "/opt/rocm")


def _hipcc():
    p = shutil.which("hipcc") or os.path.join(_rocm(), "bin", "hipcc")
    return p


def _deps_newer(target: Path, sources) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    headers = list((CSRC / "include").glob("*.h")) + list(CSRC.glob("**/*.h"))
    for s in list(sources) + headers:
        if Path(s).stat().st_mtime > t:
            return True
    return False


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(map(str, cmd)) + "\n" + r.stdout)
    return r.stdout


def _compile_hip(src: Path, force: bool) -> Path:
    obj = OBJDIR / (src.stem + (".hip.o" if src.suffix == ".hip" else ".cpp.o"))
    if force or _deps_newer(obj, [src]):
        cmd = [_hipcc(), "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
               "-I", str(CSRC / "include"), "-Wno-unused-result", "-c", str(src), "-o", str(obj)]
        if src.suffix != ".hip":
            cmd.insert(1, "-x")
            cmd.insert(2, "hip")
        _run(cmd)
    return obj


def _compile_host(src: Path, force: bool, extra=(), objdir: Path | None = None, cxx="g++") -> Path:
    obj = (objdir or OBJDIR) / (src.parent.name + "_" + src.stem + ".host.o")
    if force or _deps_newer(obj, [src]):
        cmd = [cxx, "-O2", "-fPIC", "-std=c++17", "-Wall", "-I", str(CSRC / "include"),
               *extra, "-c", str(src), "-o", str(obj)]
        _run(cmd)
    return obj


def build_hip(force=False, jobs=8) -> Path:
    LIBDIR.mkdir(parents=True, exist_ok=True)
    OBJDIR.mkdir(parents=True, exist_ok=True)
    out = LIBDIR / "libtde_hip.so"
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile_hip(s, force), HIP_SOURCES))
    if force or _deps_newer(out, objs):
        rocm = _rocm()
        _run([_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *map(str, objs), "-o", str(out),
              f"-L{rocm}/lib", "-lrccl", "-lamdhip64", f"-Wl,-rpath,{rocm}/lib",
              "-Wl,-z,defs"])   # an unresolved symbol (e.g. a kernel stub the host pass dropped) fails the build
    return out


def build_host(force=False, jobs=8, sanitize: str | None = None) -> Path:
    LIBDIR.mkdir(parents=True, exist_ok=True)
    OBJDIR.mkdir(parents=True, exist_ok=True)
    srcs = _host_sources()
    name = "libtde_host.so" if not sanitize else f"libtde_host_{sanitize}.so"
    out = LIBDIR / name
    extra = [] if not sanitize else [f"-fsanitize={sanitize}", "-g", "-O1", "-fno-omit-frame-pointer"]
    objdir = OBJDIR / sanitize if sanitize else OBJDIR
    objdir.mkdir(parents=True, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile_host(s, force, extra, objdir), srcs))
    if force or _deps_newer(out, objs):
        _run(["g++", "-shared", "-fPIC", *map(str, objs), "-o", str(out), "-lpthread", *extra])
    return out


SANITIZERS = {"address": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
              "thread": ["-fsanitize=thread"]}


def _sanitizer_cxx():
    # ROCm's LLVM ships the compiler-rt ASan / UBSan / TSan runtimes; its TSan also intercepts
    # pthread_cond_clockwait (libstdc++'s steady-clock waits), which gcc 11's libtsan misses
    # (false "double lock" reports on every timed condition-variable wait)
    c = os.path.join(_rocm(), "lib", "llvm", "bin", "clang++")
    return c if os.path.exists(c) else "g++"


def build_host_stress(sanitize: str, force=False, jobs=8) -> Path:
    """The host-runtime stress driver (csrc/tests/host_stress.cpp) linked with every host source under
    ``-fsanitize=<address|thread>``: an executable, so no sanitizer runtime has to be
    preloaded into a Python process."""
    flags = SANITIZERS[sanitize] + ["-g", "-O1", "-fno-omit-frame-pointer"]
    cxx = _sanitizer_cxx()
    objdir = OBJDIR / f"stress_{sanitize}"
    objdir.mkdir(parents=True, exist_ok=True)
    srcs = _host_sources() + [CSRC / "tests" / "host_stress.cpp"]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile_host(s, force, flags, objdir, cxx), srcs))
    out = objdir / "host_stress"
    if force or _deps_newer(out, objs):
        _run([cxx, *flags, *map(str, objs), "-o", str(out), "-lpthread"])
    return out


def build(force=False, jobs=8, hip=True, host=True):
    outs = []
    if host:
        outs.append(build_host(force, jobs))
    if hip:
        outs.append(build_hip(force, jobs))
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--no-hip", action="store_true")
    ap.add_argument("--sanitize", default=None, help="build an extra host lib with -fsanitize=<x>")
    a = ap.parse_args(argv)
    if a.sanitize:
        print(build_host(a.force, a.jobs, a.sanitize))
        return 0
    for o in build(a.force, a.jobs, hip=not a.no_hip):
        print(o)
    return 0


if __name__ == "__main__":
    sys.exit(main())
