"""In-tree build of the gfx950 kernel extension (``omnia_amd/ops/_omnia_kernels.so``).

Design: every ``csrc/*.hip`` is compiled by ``hipcc --offload-arch=gfx950`` into
an object with NO torch headers (seconds per file); only ``bindings.cpp`` sees
the torch/pybind headers.  The link is done against *torch's* bundled HIP
runtime (``torch/lib/libamdhip64.so``) so the extension and PyTorch share one
runtime instance in the process.  Objects are cached by content hash under
``omnia_amd/ops/build/`` so rebuilds only touch edited files.

Usage:  ``python -m omnia_amd.ops.build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BUILD = HERE / "build"
TARGET = HERE / "_omnia_kernels.so"
ARCH = os.environ.get("OMNIA_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = str(ROCM / "bin" / "hipcc")


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    tdir = Path(torch.__file__).resolve().parent
    incs = ce.include_paths(device_type="cuda")
    return tdir, incs


def _hash(paths, flags) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(Path(p).read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


HIP_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-ffp-contract=fast",
    "-munsafe-fp-atomics",
    "-Wno-unused-result",
]


def _compile_hip(src: Path, headers) -> Path:
    obj = BUILD / f"{src.stem}-{_hash([src, *headers], HIP_FLAGS)}.o"
    if obj.exists():
        return obj
    cmd = [HIPCC, *HIP_FLAGS, "-I", str(CSRC), "-c", str(src), "-o", str(obj)]
    subprocess.run(cmd, check=True)
    return obj


def _compile_bindings(src: Path, incs) -> Path:
    py_inc = sysconfig.get_paths()["include"]
    flags = [
        "-O2",
        "-fPIC",
        "-std=c++17",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        "-D_GLIBCXX_USE_CXX11_ABI=1",
        "-DTORCH_EXTENSION_NAME=_omnia_kernels",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-Wno-deprecated-declarations",
        "-Wno-unused-parameter",
    ]
    obj = BUILD / f"{src.stem}-{_hash([src], flags + incs)}.o"
    if obj.exists():
        return obj
    inc_flags = []
    for i in [*incs, py_inc, str(CSRC)]:
        inc_flags += ["-I", i]
    # host-only C++: clang from the ROCm toolchain, no offload
    cxx = str(ROCM / "lib" / "llvm" / "bin" / "clang++")
    cmd = [cxx, *flags, *inc_flags, "-c", str(src), "-o", str(obj)]
    subprocess.run(cmd, check=True)
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    BUILD.mkdir(exist_ok=True)
    if force:
        for f in BUILD.glob("*.o"):
            f.unlink()
    tdir, incs = _torch_paths()
    headers = sorted(CSRC.glob("*.h"))
    hip_srcs = sorted(CSRC.glob("*.hip"))
    jobs = jobs or min(8, max(1, os.cpu_count() or 1))
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile_hip, s, headers) for s in hip_srcs]
        futs.append(ex.submit(_compile_bindings, CSRC / "bindings.cpp", incs))
        objs = [f.result() for f in futs]
    for stale in set(BUILD.glob("*.o")) - set(objs):  # superseded source versions
        stale.unlink()
    tlib = tdir / "lib"
    stamp = _hash(objs, ["link"])
    stamp_file = BUILD / "link.stamp"
    if TARGET.exists() and stamp_file.exists() and stamp_file.read_text() == stamp and not force:
        return TARGET
    tmp = TARGET.with_suffix(".so.tmp")
    cmd = [
        "g++",
        "-shared",
        "-o",
        str(tmp),
        *map(str, objs),
        f"-L{tlib}",
        "-lc10",
        "-lc10_hip",
        "-ltorch",
        "-ltorch_cpu",
        "-ltorch_hip",
        "-ltorch_python",
        "-lamdhip64",
        f"-Wl,-rpath,{tlib}",
        "-Wl,--no-as-needed",
    ]
    subprocess.run(cmd, check=True)
    shutil.move(str(tmp), str(TARGET))
    stamp_file.write_text(stamp)
    if verbose:
        print(f"[omnia_amd] built {TARGET} ({len(objs)} objects, arch {ARCH})", file=sys.stderr)
    return TARGET


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.j)


if __name__ == "__main__":
    main()
