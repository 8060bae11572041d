"""In-tree build of the native engine (`mxstream/_mxs_native*.so`).

HIP sources are compiled with ``hipcc --offload-arch=gfx950`` (cross-compiles without a GPU),
host-only C++ with ``g++``; everything links into one pybind11 module next to this file so the
built object travels with the repository snapshot to the GPU box. Incremental: an object is
rebuilt only when its source, a header or the flags change.

Usage: ``python -m mxstream.build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
PKG = ROOT / "mxstream"
ARCH = os.environ.get("MXS_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = ["kernels_hip.hip", "sort_hip.hip", "parse_hip.hip", "vector_hip.hip",
               "check_hip.hip", "rolling_hist_hip.hip", "ingest_hip.hip", "listwin_hip.hip",
               "format_hip.hip", "exchange_hip.hip"]
CXX_SOURCES = ["kernels_cpu.cpp", "ingest_cpu.cpp", "runtime.cpp", "sessions.cpp", "vector_cpu.cpp",
               "vector_bindings.cpp", "trace.cpp", "check_cpu.cpp", "reader.cpp", "format.cpp", "listwin_cpu.cpp",
               "listwin_bindings.cpp", "window_tier_bindings.cpp", "window_control_bindings.cpp",
               "window_step.cpp", "window_step_bindings.cpp", "bindings.cpp"]
# roctx ranges (csrc/trace.cpp) come from the ROCm profiler SDK's marker library.
LINK_LIBS = ["-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def target_path() -> Path:
    return PKG / ("_mxs_native" + _ext_suffix())


def _includes() -> list[str]:
    import pybind11

    return [
        f"-I{CSRC}",
        f"-I{pybind11.get_include()}",
        f"-I{sysconfig.get_paths()['include']}",
    ]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    return "hipcc"


COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fvisibility=hidden",
          "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def _cmd_for(src: Path, obj: Path) -> list[str]:
    if src.suffix == ".hip":
        return [_hipcc(), f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *COMMON, *_includes(),
                "-c", str(src), "-o", str(obj)]
    # Host-only translation units: g++, no -march (the .so runs on the GPU box's CPU too).
    return ["g++", *COMMON, *_includes(), "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
            "-c", str(src), "-o", str(obj)]


def _digest(src: Path, cmd: list[str]) -> str:
    h = hashlib.sha256()
    h.update(" ".join(cmd).encode())
    h.update(src.read_bytes())
    for hdr in sorted(CSRC.glob("*.h")):
        h.update(hdr.read_bytes())
    return h.hexdigest()


def _compile(src: Path, force: bool) -> Path:
    obj = BUILD / (src.name + ".o")
    cmd = _cmd_for(src, obj)
    stamp = obj.with_suffix(".o.sha")
    dig = _digest(src, cmd)
    if not force and obj.exists() and stamp.exists() and stamp.read_text() == dig:
        return obj
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    stamp.write_text(dig)
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    """Compile every native source for gfx950 + host and link the extension module."""
    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = [CSRC / s for s in HIP_SOURCES + CXX_SOURCES]
    jobs = jobs or min(8, len(srcs))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    out = target_path()
    link = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *[str(o) for o in objs],
            *LINK_LIBS, "-o", str(out) + ".tmp"]
    newest = max(o.stat().st_mtime for o in objs)
    if force or not out.exists() or out.stat().st_mtime < newest:
        res = subprocess.run(link, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(link)}\n{res.stdout}\n{res.stderr}")
        os.replace(str(out) + ".tmp", out)
        if verbose:
            print(f"[mxstream.build] linked {out}")
    return out


SANITIZE_SOURCES = ["kernels_cpu.cpp", "vector_cpu.cpp", "tests/sanitize_main.cpp"]
SANITIZE_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                  "-fno-sanitize-recover=all"]


def build_sanitize(verbose: bool = False) -> Path:
    """Host sanitizer harness: the C++ twins + csrc/tests/sanitize_main.cpp
    under AddressSanitizer + UndefinedBehaviorSanitizer (host code only; GPU sanitizers are not
    available on the target pool). Returns the executable's path."""
    out_dir = ROOT / "build" / "sanitize"
    out_dir.mkdir(parents=True, exist_ok=True)
    exe = out_dir / "mxs_sanitize"
    srcs = [CSRC / s for s in SANITIZE_SOURCES]
    cmd = ["g++", "-std=c++17", *SANITIZE_FLAGS, f"-I{CSRC}", "-I/opt/rocm/include",
           "-D__HIP_PLATFORM_AMD__", *[str(s) for s in srcs], "-o", str(exe)]
    newest = max(s.stat().st_mtime for s in srcs + sorted(CSRC.glob("*.h")))
    if not exe.exists() or exe.stat().st_mtime < newest:
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"sanitize build failed: {' '.join(cmd)}\n{res.stderr}")
        if verbose:
            print(f"[mxstream.build] built {exe}")
    return exe


TSAN_SOURCES = ["tests/tsan_main.cpp"]
TSAN_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=thread", "-pthread"]


def build_tsan(verbose: bool = False) -> Path:
    """ThreadSanitizer harness over the threaded host code: the pinned-slot
    file reader, the socket source, the session store's spill-worker hand-off and concurrent
    key-group checkpoint writers (csrc/tests/tsan_main.cpp). Returns the executable's path."""
    out_dir = ROOT / "build" / "tsan"
    out_dir.mkdir(parents=True, exist_ok=True)
    exe = out_dir / "mxs_tsan"
    srcs = [CSRC / s for s in TSAN_SOURCES]
    cmd = ["g++", "-std=c++17", *TSAN_FLAGS, f"-I{CSRC}", "-I/opt/rocm/include",
           "-D__HIP_PLATFORM_AMD__", *[str(s) for s in srcs], "-o", str(exe)]
    newest = max(s.stat().st_mtime for s in srcs + sorted(CSRC.glob("*.h")))
    if not exe.exists() or exe.stat().st_mtime < newest:
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"tsan build failed: {' '.join(cmd)}\n{res.stderr}")
        if verbose:
            print(f"[mxstream.build] built {exe}")
    return exe


CAPI_SOURCES = ["kernels_hip.hip", "check_hip.hip", "sort_hip.hip", "rolling_hist_hip.hip",
                "vector_hip.hip", "kernels_cpu.cpp", "vector_cpu.cpp", "window_step.cpp",
                "pipeline.cpp"]


def capi_path() -> Path:
    # Next to the Python module (travels with the tree like the module; build/ does not).
    return PKG / "lib" / "libmxstream.so"


def build_capi(verbose: bool = False) -> Path:
    """The C ABI library (csrc/mxs_c.h): the native window pipeline + kernels, no Python."""
    out = capi_path()
    srcs = [CSRC / s for s in CAPI_SOURCES] + sorted(CSRC.glob("*.h"))
    if out.exists() and out.stat().st_mtime >= max(s.stat().st_mtime for s in srcs):
        return out  # up to date (also on a GPU box that received the built tree)
    BUILD.mkdir(parents=True, exist_ok=True)
    objs = [_compile(CSRC / s, False) for s in CAPI_SOURCES]
    out.parent.mkdir(parents=True, exist_ok=True)
    if not out.exists() or out.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        link = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *[str(o) for o in objs],
                "-o", str(out) + ".tmp"]
        res = subprocess.run(link, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(link)}\n{res.stdout}\n{res.stderr}")
        os.replace(str(out) + ".tmp", out)
        if verbose:
            print(f"[mxstream.build] linked {out}")
    return out


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--sanitize", action="store_true",
                    help="build the ASan/UBSan host harness (build/sanitize/mxs_sanitize)")
    ap.add_argument("--tsan", action="store_true",
                    help="build the ThreadSanitizer host harness (build/tsan/mxs_tsan)")
    ap.add_argument("--capi", action="store_true",
                    help="build the C ABI library build/lib/libmxstream.so (csrc/mxs_c.h)")
    a = ap.parse_args(argv)
    if a.capi:
        print(build_capi(verbose=True))
        return 0
    if a.sanitize:
        print(build_sanitize(verbose=True))
        return 0
    if a.tsan:
        print(build_tsan(verbose=True))
        return 0
    p = build(force=a.force, jobs=a.jobs, verbose=True)
    print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
