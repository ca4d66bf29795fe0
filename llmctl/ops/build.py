"""Build the in-tree HIP kernel library ``llmctl/ops/_llmctl_hip.so`` for gfx950.

Plain ``hipcc`` invocations (no hipify, no torch JIT cache): every ``csrc/*.hip`` /
``csrc/*.cpp`` compiles to an object under ``build/ops`` (rebuilt when the content hash of the
source, the headers or the flags changes), then one link step produces the shared library next to this file, so it
travels with the repository snapshot to the GPU box.

    python -m llmctl.ops.build [-j N] [--force] [--arch gfx950] [--save-temps]
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
OUT = HERE / "_llmctl_hip.so"
BUILD = HERE.parents[1] / "build" / "ops"


def torch_paths():
    import torch.utils.cpp_extension as ce

    return ce.include_paths(), ce.library_paths()


def hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    p = Path(rocm) / "bin" / "hipcc"
    return str(p) if p.exists() else "hipcc"


def compile_flags(arch: str, save_temps: bool = False):
    incs, _ = torch_paths()
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={arch}", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
             "-D_GLIBCXX_USE_CXX11_ABI=1", "-Wno-unused-result", "-Wno-deprecated-declarations",
             "-Wno-return-type", f"-I{CSRC}"]
    flags += [f"-I{i}" for i in incs]
    if save_temps:
        flags += ["-save-temps=obj"]
    # diagnostic builds only (e.g. LLMCTL_BUILD_DEFINES="LLMCTL_STAMP LLMCTL_STAMP_EXP=2" for the
    # persistent GEMM's cycle stamps, tools/gemm_stamps.py); the production library sets none
    flags += [f"-D{d}" for d in os.environ.get("LLMCTL_BUILD_DEFINES", "").split() if d]
    return flags


# per-source extra flags.  flash_attn_bwd: MFMA results in the VGPR form — by default hipcc gave
# the S / dP products AGPR destinations (occupancy-1 kernel, AGPRs free) and then moved every
# element back with v_accvgpr_read for the softmax VALU (~120 moves per tile); the dK/dV
# accumulators are pinned to AGPRs by their inline-asm MFMAs instead.
FILE_FLAGS = {"flash_attn_bwd.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-fno-slp-vectorize"]}


def file_flags(src: Path, flags):
    return flags + FILE_FLAGS.get(src.name, [])


def _digest(src: Path, flags) -> str:
    """Content key of one object: the source, every csrc header and the compile flags (not
    mtimes: a restored or copied tree can carry stale objects with newer timestamps)."""
    import hashlib

    h = hashlib.sha256()
    for d in [src] + sorted(list(CSRC.glob("*.h")) + list(CSRC.glob("*.inc"))):
        h.update(d.name.encode())
        h.update(d.read_bytes())
    h.update("\0".join(flags).encode())
    return h.hexdigest()


def _needs(src: Path, obj: Path, flags) -> bool:
    key = obj.with_suffix(obj.suffix + ".key")
    return not (obj.exists() and key.exists() and key.read_text() == _digest(src, flags))


def build(arch: str = "gfx950", jobs: int = 0, force: bool = False, save_temps: bool = False, verbose: bool = True) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))
    flags = compile_flags(arch, save_temps)
    todo = []
    objs = []
    for s in srcs:
        o = BUILD / (s.name + ".o")
        objs.append(o)
        if force or _needs(s, o, file_flags(s, flags)):
            todo.append((s, o))

    def _one(so):
        s, o = so
        cmd = [hipcc()] + file_flags(s, flags) + ["-c", str(s), "-o", str(o)]
        key = _digest(s, file_flags(s, flags))  # before compiling: a source edited mid-build stays stale
        r = subprocess.run(cmd, capture_output=True, text=True, cwd=str(BUILD))
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {s.name}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        o.with_suffix(o.suffix + ".key").write_text(key)
        return s.name

    jobs = jobs or min(8, max(1, (os.cpu_count() or 4)))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for name in ex.map(_one, todo):
                if verbose:
                    print(f"[llmctl.ops.build] compiled {name}", flush=True)
    relink = force or bool(todo) or not OUT.exists() or any(o.stat().st_mtime > OUT.stat().st_mtime for o in objs)
    if relink:
        _, libs = torch_paths()
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={arch}", "-o", str(OUT)] + [str(o) for o in objs]
        for L in libs:
            cmd += [f"-L{L}", f"-Wl,-rpath,{L}"]
        cmd += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[llmctl.ops.build] linked {OUT}", flush=True)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default=os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0])
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--save-temps", action="store_true")
    a = ap.parse_args(argv)
    build(a.arch, a.jobs, a.force, a.save_temps)


if __name__ == "__main__":
    main()
