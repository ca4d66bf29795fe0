"""Build the native host runtime extension in-tree (g++ -O3 + pybind11).

    python -m llmctl.native.build [--force] [--sanitize]

``--sanitize`` (or ``LLMCTL_SANITIZE=1``) builds the host runtime with AddressSanitizer +
UndefinedBehaviorSanitizer (host code only — GPU ASan is not available on the MI355X pool);
run it under ``LD_PRELOAD=$(g++ -print-file-name=libasan.so)``.  The concurrency-heavy parts
(prefetching token loader, block allocator) are additionally exercised by ThreadSanitizer
with ``--sanitize=thread``.
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


def build(force: bool = False, verbose: bool = True, sanitize: str = "", out: Path = None) -> Path:
    import os

    import pybind11

    sanitize = sanitize or ("address" if os.environ.get("LLMCTL_SANITIZE") == "1" else "")
    out = out or out_path()
    if not force and not sanitize and out.exists() and out.stat().st_mtime > SRC.stat().st_mtime:
        return out
    inc = sysconfig.get_paths()["include"]
    san = []
    if sanitize == "address":
        san = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined"]
    elif sanitize == "thread":
        san = ["-O1", "-g", "-fsanitize=thread"]
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-result", "-pthread", *san,
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
    ap.add_argument("--sanitize", nargs="?", const="address", default="", choices=["", "address", "thread"])
    ap.add_argument("--out", type=Path, default=None)
    a = ap.parse_args()
    build(a.force, sanitize=a.sanitize, out=a.out)
    sys.exit(0)
