"""``DistModule``: the reference's data-parallel model wrapper (``dist_helper.py:369-439``) re-designed
around the bucketed reducer.

* construction broadcasts every state tensor from rank 0 as one flat buffer per dtype;
* gradients live in flat buckets and are all-reduced asynchronously while backward is still running
  (post-accumulate-grad hooks, :class:`GradientReducer`), so ``sync_gradients()`` only waits for the
  tail bucket -- the reference issues one blocking all-reduce per parameter after backward;
* forwards and the model API (``forward``, ``sl_train``, ``rl_learner_forward``, ``compute_*``,
  ``state_dict``...) are delegated to the wrapped module, and the state-dict keys carry no
  ``module.`` prefix, so checkpoints are interchangeable with single-process runs.
"""
from __future__ import annotations

import torch.nn as nn

from . import dist as pdist
from .dp import GradientReducer


class DistModule(nn.Module):
    def __init__(self, module: nn.Module, bucket_mb: float = 32.0, comm_dtype=None, group=None,
                 sync: bool = True):
        super().__init__()
        self.module = module
        pdist.broadcast_module(module)
        # sync=False in the reference registers (broken) per-parameter async hooks; here overlap is
        # always on and sync only selects whether sync_gradients() blocks until the buckets are done
        self.reducer = GradientReducer(module.parameters(), bucket_mb=bucket_mb, comm_dtype=comm_dtype,
                                       group=group)
        self.sync = sync

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.module, name)

    def zero_grad(self, set_to_none: bool = False):
        self.reducer.zero_grad()

    def sync_gradients(self):
        self.reducer.synchronize()

    def broadcast_params(self):
        pdist.broadcast_module(self.module)

    def state_dict(self, *args, **kwargs):
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict: bool = True):
        sd = {k[7:] if k.startswith('module.') else k: v for k, v in state_dict.items()}
        return self.module.load_state_dict(sd, strict=strict)

    def named_parameters(self, *args, **kwargs):
        return self.module.named_parameters(*args, **kwargs)

    def parameters(self, recurse: bool = True):
        return self.module.parameters(recurse)
