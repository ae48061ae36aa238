"""Process-group setup and small collectives for one-process-per-GPU training over RCCL/xGMI.

Replaces the reference's ``dist_helper`` (``distar/ctools/utils/dist_helper.py:259-366``) with the
MI355X-first pattern:

* ``init()`` reads RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* (torchrun) or explicit args
  (``--init_method tcp://... --rank --world_size`` like ``rl_train.py``), binds ``cuda:local_rank``
  and creates the process group (backend ``nccl`` == RCCL on ROCm, ``gloo`` on CPU);
* parameters/buffers are broadcast as ONE flat buffer per dtype (the reference broadcasts 432-515
  tensors one by one);
* log scalars are all-reduced as ONE packed vector per step (the reference issues ~43 one-element
  all-reduces and a CPU-tensor broadcast that NCCL rejects).
"""
from __future__ import annotations

import datetime
import os
from typing import Dict, Iterable, List, Optional

import torch
import torch.distributed as dist


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def get_rank() -> int:
    return dist.get_rank() if is_initialized() else 0


def get_world_size() -> int:
    return dist.get_world_size() if is_initialized() else 1


def get_local_rank() -> int:
    return int(os.environ.get('LOCAL_RANK', get_rank() % max(torch.cuda.device_count(), 1)))


def init(backend: Optional[str] = None, init_method: Optional[str] = None, rank: Optional[int] = None,
         world_size: Optional[int] = None, timeout_s: int = 1800) -> tuple:
    """Initialise the default process group if the environment asks for one.  Returns (rank, world)."""
    if is_initialized():
        return get_rank(), get_world_size()
    env_world = int(os.environ.get('WORLD_SIZE', '1'))
    world_size = env_world if world_size is None else world_size
    if world_size <= 1 and init_method is None:
        return 0, 1
    rank = int(os.environ.get('RANK', '0')) if rank is None else rank
    # surface a dead / hung peer as an error after `timeout_s` instead of a silent hang (RCCL honours it)
    os.environ.setdefault('TORCH_NCCL_ASYNC_ERROR_HANDLING', '1')
    use_gpu = torch.cuda.is_available()
    if backend is None:
        backend = 'nccl' if use_gpu else 'gloo'
    if use_gpu:
        torch.cuda.set_device(get_local_rank() if 'LOCAL_RANK' in os.environ else rank % torch.cuda.device_count())
    kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
    if init_method is not None:
        kw.update(init_method=init_method, rank=rank, world_size=world_size)
    else:
        kw.update(rank=rank, world_size=world_size)
    if backend == 'nccl' and use_gpu:
        kw['device_id'] = torch.device('cuda', torch.cuda.current_device())
    dist.init_process_group(**kw)
    return rank, world_size


def finalize():
    if is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def barrier():
    if is_initialized():
        if dist.get_backend() == 'nccl':
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def _flat_groups(tensors: Iterable[torch.Tensor]) -> Dict[tuple, List[torch.Tensor]]:
    groups: Dict[tuple, List[torch.Tensor]] = {}
    for t in tensors:
        groups.setdefault((t.dtype, t.device), []).append(t)
    return groups


@torch.no_grad()
def broadcast_tensors(tensors: Iterable[torch.Tensor], src: int = 0) -> None:
    """Broadcast every tensor from ``src`` using one flat buffer per (dtype, device)."""
    if get_world_size() == 1:
        return
    for _, ts in _flat_groups(tensors).items():
        flat = torch.cat([t.reshape(-1) for t in ts])
        dist.broadcast(flat, src)
        off = 0
        for t in ts:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n


def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    broadcast_tensors(list(module.state_dict().values()), src)


def allreduce_scalars(values: Dict[str, torch.Tensor], average: bool = True) -> Dict[str, torch.Tensor]:
    """All-reduce a dict of 0-d tensors with ONE collective; returns a dict of host floats."""
    if not values:
        return {}
    keys = sorted(values)
    first = next(iter(values.values()))
    if is_initialized() and dist.get_backend() == 'nccl':
        dev = torch.device('cuda', torch.cuda.current_device())
    else:
        dev = first.device if torch.is_tensor(first) else torch.device('cpu')
    vec = torch.stack([torch.as_tensor(values[k], dtype=torch.float32, device=dev).reshape(()) for k in keys])
    if get_world_size() > 1:
        dist.all_reduce(vec)
        if average:
            vec /= get_world_size()
    host = vec.cpu().tolist()
    return dict(zip(keys, host))


def broadcast_object(obj, src: int = 0):
    if get_world_size() == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src)
    return lst[0]
