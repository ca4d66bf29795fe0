"""Build the native host runtime extension in-tree (g++ -O3 + pybind11).

    python -m llmctl.native.build [--force]
"""

from __future__ import annotations

import argparse
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "csrc" / "runtime.cpp"


def out_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return HERE / f"_llmctl_native{suffix}"


def build(force: bool = False, verbose: bool = True) -> Path:
    import pybind11

    out = out_path()
    if not force and out.exists() and out.stat().st_mtime > SRC.stat().st_mtime:
        return out
    inc = sysconfig.get_paths()["include"]
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-result", "-pthread",
           f"-I{pybind11.get_include()}", f"-I{inc}", str(SRC), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n{' '.join(cmd)}\n{r.stderr}")
    if verbose:
        print(f"[llmctl.native.build] built {out}", flush=True)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    build(a.force)
    sys.exit(0)
