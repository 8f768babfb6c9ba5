"""Build the host-native extension ``omnia_amd/native/_omnia_native*.so`` in-tree.

``python -m omnia_amd.native.build``  (g++, pybind11 headers; objects cached by
content hash like the HIP build)."""
from __future__ import annotations

import hashlib
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
TARGET = HERE / ("_omnia_native" + sysconfig.get_config_var("EXT_SUFFIX"))
FLAGS = ["-O2", "-std=c++17", "-fPIC", "-shared", "-maes", "-mpclmul", "-mssse3", "-msse4.1",
         "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]


def build(force: bool = False) -> Path:
    import pybind11

    srcs = sorted(CSRC.glob("*.cpp"))
    h = hashlib.sha256()
    for s in srcs:
        h.update(s.read_bytes())
    h.update(" ".join(FLAGS).encode())
    stamp = HERE / ".build_hash"
    digest = h.hexdigest()
    if not force and TARGET.exists() and stamp.exists() and stamp.read_text() == digest:
        return TARGET
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    cmd = ["g++", *FLAGS, *inc, *map(str, srcs), "-o", str(TARGET)]
    subprocess.run(cmd, check=True)
    stamp.write_text(digest)
    print(f"[omnia_amd] built {TARGET}")
    return TARGET


if __name__ == "__main__":
    build("--force" in sys.argv)
