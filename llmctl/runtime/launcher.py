"""Launchers and process orchestration (the process boundary between CLI and workers).

Reference: ``llmctl/runtime/launcher.py:21-332`` (LaunchConfig, Local/Slurm/MPI launchers,
``create_launcher``, ``ProcessOrchestrator``).  Same API, ROCm-native environment:

* ``HIP_VISIBLE_DEVICES`` instead of ``CUDA_VISIBLE_DEVICES``; RCCL honours ``NCCL_*``;
* ``HSA_ENABLE_IPC_MODE_LEGACY=0`` is propagated (dmabuf IPC; required by RCCL here);
* determinism -> ``HIP_LAUNCH_BLOCKING=1`` + ``PYTHONHASHSEED`` (ref ``launcher.py:86-90``);
* ``k8s`` (advertised by the reference, ``train.py:23``, but unsupported there) renders an
  indexed Job manifest;
* MPI maps ``OMPI_COMM_WORLD_*`` to torch env vars inside the worker (the reference set
  ``OMPI_COMM_WORLD_RANK=0`` in the *parent*);
* elastic restarts: ``max_restarts`` is forwarded to torchrun and the orchestrator can
  auto-resume from ``<output_dir>/latest``.

Launchers never exec in the caller: they return a ``Popen`` of a child process (the GPU
box forbids exec from processes that touched the GPU).
"""

from __future__ import annotations

import os
import shlex
import signal
import subprocess
import sys
import tempfile
import time
from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional


@dataclass
class LaunchConfig:
    nodes: int = 1
    gpus_per_node: int = 1
    cpus_per_task: Optional[int] = None
    mixed_precision: str = "bf16"
    launcher: str = "local"
    backend: str = "nccl"  # "nccl" == RCCL on ROCm
    config_path: Optional[str] = None
    data_path: Optional[str] = None
    plan_path: Optional[str] = None
    checkpoint_path: Optional[str] = None
    seed: int = 42
    deterministic: bool = False
    log_level: str = "info"
    gradient_accumulation_steps: int = 1
    gradient_clipping: float = 1.0
    master_addr: str = "127.0.0.1"
    master_port: int = field(default_factory=lambda: int(os.environ.get("LLMCTL_MASTER_PORT", "29500")))
    node_rank: int = 0
    max_restarts: int = 0
    debug: bool = False  # race/fault hunting: serialized kernels, blocking collectives, verbose RCCL
    extra_env: Dict[str, str] = field(default_factory=dict)

    def total_gpus(self) -> int:
        return self.nodes * self.gpus_per_node


class BaseLauncher(ABC):
    def __init__(self, config: LaunchConfig):
        self.config = config

    @abstractmethod
    def launch(self, script_path: str, script_args: List[str]) -> subprocess.Popen:
        ...

    def build_command(self, script_path: str, script_args: List[str]) -> List[str]:
        raise NotImplementedError

    def get_environment(self) -> Dict[str, str]:
        c = self.config
        env = os.environ.copy()
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        env["LLMCTL_LOG_LEVEL"] = c.log_level
        env["PYTHONUNBUFFERED"] = "1"
        if c.deterministic:
            env["PYTHONHASHSEED"] = str(c.seed)
            env["HIP_LAUNCH_BLOCKING"] = "1"
            env["LLMCTL_DETERMINISTIC"] = "1"
        if c.debug or os.environ.get("LLMCTL_DEBUG") == "1":
            # every kernel completes before the next is launched (a fault points at its kernel),
            # collectives block with the timeout (a hang becomes an error on the rank that hung)
            env["AMD_SERIALIZE_KERNEL"] = "3"
            env["AMD_SERIALIZE_COPY"] = "3"
            env["HIP_LAUNCH_BLOCKING"] = "1"
            env["TORCH_NCCL_BLOCKING_WAIT"] = "1"
            env["NCCL_DEBUG"] = "INFO"
            env["LLMCTL_STREAM_CHECK"] = "1"
        repo_root = str(Path(__file__).resolve().parents[2])
        env["PYTHONPATH"] = repo_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        env.update(c.extra_env)
        return env


class LocalLauncher(BaseLauncher):
    """torchrun on this node (ref ``launcher.py:65-120``)."""

    def get_environment(self) -> Dict[str, str]:
        env = super().get_environment()
        c = self.config
        env["WORLD_SIZE"] = str(c.total_gpus())
        env["NPROC_PER_NODE"] = str(c.gpus_per_node)
        env["MASTER_ADDR"] = c.master_addr
        env["MASTER_PORT"] = str(c.master_port)
        if "HIP_VISIBLE_DEVICES" not in os.environ and "ROCR_VISIBLE_DEVICES" not in os.environ:
            env["HIP_VISIBLE_DEVICES"] = ",".join(str(i) for i in range(c.gpus_per_node))
        env.setdefault("NCCL_DEBUG", "WARN")
        return env

    def build_command(self, script_path: str, script_args: List[str]) -> List[str]:
        c = self.config
        cmd = [sys.executable, "-m", "torch.distributed.run", f"--nproc_per_node={c.gpus_per_node}",
               f"--nnodes={c.nodes}", f"--node_rank={c.node_rank}", f"--master_addr={c.master_addr}",
               f"--master_port={c.master_port}"]
        if c.max_restarts:
            cmd.append(f"--max_restarts={c.max_restarts}")
        if script_path.endswith(".py"):
            cmd.append(script_path)
        else:
            cmd += ["-m", script_path]
        return cmd + list(script_args)

    def launch(self, script_path: str, script_args: List[str]) -> subprocess.Popen:
        return subprocess.Popen(self.build_command(script_path, script_args), env=self.get_environment(),
                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, bufsize=1,
                                start_new_session=True)


class SlurmLauncher(BaseLauncher):
    """sbatch script, one task per GPU (ref ``launcher.py:122-192``)."""

    def get_environment(self) -> Dict[str, str]:
        env = super().get_environment()
        env.setdefault("NCCL_DEBUG", "WARN")
        return env

    def create_slurm_script(self, script_path: str, script_args: List[str]) -> str:
        c = self.config
        mod = script_path if not script_path.endswith(".py") else None
        target = f"-m {mod}" if mod else shlex.quote(script_path)
        cpus = f"#SBATCH --cpus-per-task={c.cpus_per_task}\n" if c.cpus_per_task else ""
        return f"""#!/bin/bash
#SBATCH --job-name=llmctl-train
#SBATCH --nodes={c.nodes}
#SBATCH --ntasks-per-node={c.gpus_per_node}
#SBATCH --gpus-per-node={c.gpus_per_node}
{cpus}#SBATCH --time=24:00:00
export MASTER_ADDR=$(scontrol show hostnames "$SLURM_JOB_NODELIST" | head -n 1)
export MASTER_PORT={c.master_port}
export WORLD_SIZE=$SLURM_NTASKS
export HSA_ENABLE_IPC_MODE_LEGACY=0
srun bash -c 'RANK=$SLURM_PROCID LOCAL_RANK=$SLURM_LOCALID {shlex.quote(sys.executable)} {target} {" ".join(shlex.quote(a) for a in script_args)}'
"""

    def build_command(self, script_path: str, script_args: List[str]) -> List[str]:
        fd, path = tempfile.mkstemp(suffix=".sbatch", prefix="llmctl-")
        with os.fdopen(fd, "w") as f:
            f.write(self.create_slurm_script(script_path, script_args))
        return ["sbatch", path]

    def launch(self, script_path: str, script_args: List[str]) -> subprocess.Popen:
        return subprocess.Popen(self.build_command(script_path, script_args), env=self.get_environment(),
                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


class MPILauncher(BaseLauncher):
    """mpirun; ranks come from ``OMPI_COMM_WORLD_*`` mapped in the worker (ref ``:194-236``)."""

    def build_command(self, script_path: str, script_args: List[str]) -> List[str]:
        c = self.config
        target = ["-m", script_path] if not script_path.endswith(".py") else [script_path]
        return ["mpirun", "-np", str(c.total_gpus()), "--bind-to", "none", "--map-by", "slot",
                "-x", "NCCL_DEBUG", "-x", "PYTHONPATH", "-x", "HSA_ENABLE_IPC_MODE_LEGACY",
                "-x", f"MASTER_ADDR={c.master_addr}", "-x", f"MASTER_PORT={c.master_port}",
                sys.executable] + target + list(script_args)

    def launch(self, script_path: str, script_args: List[str]) -> subprocess.Popen:
        env = self.get_environment()
        env.setdefault("NCCL_DEBUG", "WARN")
        return subprocess.Popen(self.build_command(script_path, script_args), env=env, stdout=subprocess.PIPE,
                                stderr=subprocess.STDOUT, text=True)


class K8sLauncher(BaseLauncher):
    """Indexed Job manifest applied with kubectl (one pod per node, torchrun inside)."""

    def render_manifest(self, script_path: str, script_args: List[str], image: str = "llmctl:rocm") -> str:
        c = self.config
        args = " ".join(shlex.quote(a) for a in script_args)
        target = f"-m {script_path}" if not script_path.endswith(".py") else script_path
        return f"""apiVersion: batch/v1
kind: Job
metadata: {{name: llmctl-train}}
spec:
  completionMode: Indexed
  completions: {c.nodes}
  parallelism: {c.nodes}
  template:
    spec:
      restartPolicy: Never
      containers:
      - name: worker
        image: {image}
        env: [{{name: HSA_ENABLE_IPC_MODE_LEGACY, value: "0"}}, {{name: MASTER_PORT, value: "{c.master_port}"}}]
        resources: {{limits: {{amd.com/gpu: {c.gpus_per_node}}}}}
        command: ["bash", "-c", "python -m torch.distributed.run --nnodes={c.nodes} --nproc_per_node={c.gpus_per_node} --node_rank=$JOB_COMPLETION_INDEX --master_addr=llmctl-train-0.llmctl-train --master_port={c.master_port} {target} {args}"]
"""

    def build_command(self, script_path: str, script_args: List[str]) -> List[str]:
        fd, path = tempfile.mkstemp(suffix=".yaml", prefix="llmctl-k8s-")
        with os.fdopen(fd, "w") as f:
            f.write(self.render_manifest(script_path, script_args))
        return ["kubectl", "apply", "-f", path]

    def launch(self, script_path: str, script_args: List[str]) -> subprocess.Popen:
        return subprocess.Popen(self.build_command(script_path, script_args), env=self.get_environment(),
                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def create_launcher(config: LaunchConfig) -> BaseLauncher:
    kinds = {"local": LocalLauncher, "slurm": SlurmLauncher, "mpi": MPILauncher, "k8s": K8sLauncher}
    if config.launcher not in kinds:
        raise ValueError(f"Unsupported launcher: {config.launcher} (choose from {sorted(kinds)})")
    return kinds[config.launcher](config)


class ProcessOrchestrator:
    """Start / monitor / stop training (ref ``launcher.py:249-332``) plus auto-resume:
    on a non-zero exit with ``restarts_left`` it relaunches with
    ``--resume-from-checkpoint <output_dir>``."""

    def __init__(self, config: LaunchConfig, echo=print):
        self.config = config
        self.launcher = create_launcher(config)
        self.process: Optional[subprocess.Popen] = None
        self.echo = echo
        self.restarts = 0

    def start_training(self, script_path: str, script_args: List[str], auto_resume_dir: Optional[str] = None,
                       restarts: int = 0) -> int:
        args = list(script_args)
        while True:
            self.process = self.launcher.launch(script_path, args)
            rc = self._monitor()
            if rc == 0 or self.restarts >= restarts or auto_resume_dir is None:
                return rc
            self.restarts += 1
            latest = Path(auto_resume_dir) / "latest"
            if latest.exists() and "--resume-from-checkpoint" not in args:
                args += ["--resume-from-checkpoint", str(Path(auto_resume_dir) / latest.read_text().strip())]
            self.echo(f"[orchestrator] exit code {rc}; restart {self.restarts}/{restarts}")

    def _monitor(self) -> int:
        p = self.process
        assert p is not None
        if p.stdout is not None:
            for line in p.stdout:
                self.echo(line.rstrip("\n"))
        return p.wait()

    def stop_training(self) -> None:
        p = self.process
        if p is None or p.poll() is not None:
            return
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except Exception:
            p.terminate()
        try:
            p.wait(timeout=5)
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except Exception:
                p.kill()

    def get_status(self) -> Dict[str, object]:
        p = self.process
        if p is None:
            return {"status": "not_started"}
        rc = p.poll()
        return {"status": "running" if rc is None else "finished", "returncode": rc, "pid": p.pid,
                "restarts": self.restarts}
