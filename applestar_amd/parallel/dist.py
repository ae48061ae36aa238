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


def local_device_index() -> int:
    """This rank's GPU: LOCAL_RANK modulo the visible devices (several gloo ranks can share one GPU)."""
    return get_local_rank() % max(torch.cuda.device_count(), 1)


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
        # APPLESTAR_DIST_BACKEND=gloo rehearses the multi-rank GPU path with several ranks sharing one GPU
        # (RCCL needs one GPU per rank)
        backend = os.environ.get('APPLESTAR_DIST_BACKEND') or ('nccl' if use_gpu else 'gloo')
    if use_gpu:
        local = get_local_rank() if 'LOCAL_RANK' in os.environ else rank
        torch.cuda.set_device(local % torch.cuda.device_count())
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


# ---------------------------------------------------------------------------------------------- extras
def allreduce(x: torch.Tensor, average: bool = True, group=None) -> torch.Tensor:
    """In-place all-reduce (``dist_helper.py:272-289``); AVG is done inside RCCL on the nccl backend."""
    if not is_initialized() or dist.get_world_size(group) == 1:
        return x
    if average and dist.get_backend(group) == 'nccl':
        dist.all_reduce(x, op=dist.ReduceOp.AVG, group=group)
    else:
        dist.all_reduce(x, group=group)
        if average:
            x.div_(dist.get_world_size(group))
    return x


def broadcast(x: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    if is_initialized():
        dist.broadcast(x, src, group=group)
    return x


def simple_group_split(world_size: int, rank: int, num_groups: int):
    """Create ``num_groups`` process groups of consecutive ranks (every rank must call this with the same
    arguments, as ``new_group`` is collective) and return the one containing ``rank``
    (``dist_helper.py:292-366``)."""
    assert world_size % num_groups == 0, (world_size, num_groups)
    size = world_size // num_groups
    groups = [dist.new_group(list(range(i * size, (i + 1) * size))) for i in range(num_groups)]
    return groups[rank // size]


def get_group(group_size: int):
    """Process group of ``group_size`` consecutive ranks containing this rank (None when not distributed)."""
    if not is_initialized():
        return None
    world = get_world_size()
    return simple_group_split(world, get_rank(), world // group_size)


def _slurm_master(nodelist: str) -> str:
    """First host of a SLURM nodelist such as ``node[03-05,07],gpu1`` -> ``node03``."""
    head = nodelist.split(',')[0] if '[' not in nodelist.split(',')[0] else nodelist[:nodelist.index(']') + 1]
    if '[' in head:
        prefix, rng = head.split('[', 1)
        first = rng.rstrip(']').split(',')[0].split('-')[0]
        return prefix + first
    return head


def init_from_method(method: str = 'torch', port: int = 29500, backend: Optional[str] = None) -> tuple:
    """``dist_init(method)`` of the reference (``dist_helper.py:321-344``): 'torch' (torchrun env),
    'single_node' (RANK/WORLD_SIZE with 127.0.0.1) or 'slurm' (SLURM_PROCID/SLURM_NTASKS/SLURM_LOCALID,
    master = first node of SLURM_NODELIST)."""
    if method == 'slurm':
        os.environ.setdefault('RANK', os.environ['SLURM_PROCID'])
        os.environ.setdefault('WORLD_SIZE', os.environ['SLURM_NTASKS'])
        os.environ.setdefault('LOCAL_RANK', os.environ.get('SLURM_LOCALID', '0'))
        os.environ.setdefault('MASTER_ADDR', _slurm_master(os.environ.get('SLURM_NODELIST', '127.0.0.1')))
        os.environ.setdefault('MASTER_PORT', str(port))
    elif method == 'single_node':
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', str(port))
    elif method != 'torch':
        raise ValueError(f'unknown dist init method {method!r}')
    return init(backend=backend)
