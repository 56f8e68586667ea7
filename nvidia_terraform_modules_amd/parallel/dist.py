"""One-process-per-GPU bootstrap for torch.distributed over RCCL (xGMI).

On ROCm the ``"nccl"`` backend IS RCCL. The CPU test path uses ``gloo`` with the
same code. Rendezvous always uses the env contract of ``torch.distributed.run``
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT); the default
MASTER_ADDR is 127.0.0.1 because container hostnames may not resolve.

Reference parity: the reference has no collective code at all; its only
multi-node enabler is the all-protocol node<->node security-group rule
(/root/reference/eks/main.tf:29-48), reproduced in ``eks/main.tf``.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as tdist


@dataclass(frozen=True)
class DistEnv:
    rank: int
    local_rank: int
    world_size: int
    backend: str
    device: torch.device

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init(backend: str | None = None, device_type: str | None = None) -> DistEnv:
    """Initialise (or reuse) the default process group from the env contract.

    ``backend`` defaults to ``nccl`` (RCCL) when GPUs are present, ``gloo``
    otherwise. world_size == 1 never creates a process group. Collectives time
    out after ``NTM_DIST_TIMEOUT_S`` seconds (default 300, not torch's 10 min):
    a rank that never arrives fails the job quickly instead of holding the node.
    """
    world = env_int("WORLD_SIZE", 1)
    rank = env_int("RANK", 0)
    local = env_int("LOCAL_RANK", rank)
    use_gpu = device_type == "cuda" if device_type else torch.cuda.is_available()
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    if use_gpu:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not tdist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        kwargs = {"timeout": datetime.timedelta(seconds=env_int("NTM_DIST_TIMEOUT_S", 300))}
        if backend == "nccl":
            kwargs["device_id"] = device
        tdist.init_process_group(backend=backend, rank=rank, world_size=world, **kwargs)
    return DistEnv(rank=rank, local_rank=local, world_size=world, backend=backend, device=device)


def barrier(env: DistEnv) -> None:
    if env.world_size > 1:
        if env.backend == "nccl":
            tdist.barrier(device_ids=[env.local_rank])
        else:
            tdist.barrier()


def all_reduce_max(env: DistEnv, value: float) -> float:
    if env.world_size == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=env.device if env.backend == "nccl" else "cpu")
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum(env: DistEnv, value: float) -> float:
    if env.world_size == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=env.device if env.backend == "nccl" else "cpu")
    tdist.all_reduce(t, op=tdist.ReduceOp.SUM)
    return float(t.item())


def all_gather_obj(env: DistEnv, obj) -> list:
    if env.world_size == 1:
        return [obj]
    out = [None] * env.world_size
    tdist.all_gather_object(out, obj)
    return out


def shutdown(env: DistEnv) -> None:
    if env.world_size > 1 and tdist.is_initialized():
        tdist.destroy_process_group()
