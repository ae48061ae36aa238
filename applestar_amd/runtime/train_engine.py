"""The learner step machinery shared by the RL and SL trainers (rl/trainer.py, sl/trainer.py).

Reference: ``distar/ctools/worker/learner/base_learner.py`` + ``distar/agent/default/rl_learner.py:82-145`` and
``sl_learner.py:46-77`` each build their own model / optimizer / clip / all-reduce; the two learners differ only
in the forward + loss and in the optimizer's hyper-parameters.  Here everything between "the loss exists" and
"the weights changed" lives in ONE class, so every optimisation of that path applies to both learners:

* device setup: NHWC (channels_last) convolutions, MIOpen autotuning opt-in, weights broadcast from rank 0;
* precision: fp32 (the default, like-for-like with the reference) or bf16 compute weights backed by fp32
  master weights in one flat buffer (parallel/mixed.py);
* derived weight forms (transposed GEMM weights, flipped conv weights, fp32 biases) rebuilt once per
  optimizer step in a few multi-tensor launches (ops/native.py ``DerivedWeights``), in both precisions;
* backward straight into the flat gradient buckets (parallel/dp.py) and one bucketed RCCL reduction;
* clip + Adam as two (pytorch_norm) or three (momentum_norm) native launches (utils/fused_optim.py,
  csrc/kernels/optim.hip), with the step's hyper-parameters in a device buffer so the update can be replayed
  from a HIP graph;
* the LSTM-exchange health gate: the split LSTM recurrence raises a device flag when its cross-workgroup
  exchange times out; the flag is MIN-reduced across ranks together with the gradients, so EVERY rank skips
  the same step (a rank-local skip would let the replicas' weights diverge), and the fused update returns
  before touching the weights or the optimizer state.
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, Optional

import torch

from ..parallel import dist as pdist
from ..parallel.dp import GradientReducer
from ..parallel.mixed import MasterWeights
from ..utils.grad_clip import build_grad_clip
from ..utils.optim import build_optimizer

FUSED_CLIP_ADAM = os.environ.get('APPLESTAR_FUSED_ADAM', '1') != '0'     # A/B switch

# grad-clip types whose state is all on the device (safe to replay from a graph)
GRAPH_SAFE_CLIPS = ('none', 'pytorch_norm', 'clip_norm', 'clip_const', 'momentum_norm')


def amp_context(device: torch.device, dtype_name: Optional[str]):
    if device.type != 'cuda' or not dtype_name:
        return contextlib.nullcontext()
    # no autocast weight cache: the compute weights are already bf16 (master weights), and a cache
    # must not outlive a HIP-graph capture
    return torch.autocast('cuda', dtype=getattr(torch, dtype_name), cache_enabled=False)


class TrainEngine:
    """Base of :class:`~applestar_amd.rl.trainer.RLTrainer` / :class:`~applestar_amd.sl.trainer.SLTrainer`.

    Subclasses set ``self.cfg`` (with a ``learner`` section), build ``self.model`` and call
    :meth:`_setup_engine`; a step is then ``backward(loss)`` -> ``_reduce()`` -> ``_update()``."""

    # optimizer hyper-parameters of the learner (the reference's RL learner: betas (0, 0.99), eps 1e-5)
    ADAM_BETAS = (0.9, 0.999)
    ADAM_EPS = 1e-8

    def _setup_engine(self, device):
        lc = self.cfg.learner
        self.device = torch.device(device)
        self.model.to(self.device)
        if self.device.type == 'cuda':
            # MIOpen find-mode autotuning (cudnn.benchmark) is opt-in: it measured ~10% faster convs on the
            # bench shapes, but two runs that used it left the GPU in a memory-fault state
            torch.backends.cudnn.benchmark = bool(lc.get('conv_autotune', False))
            # NHWC convolutions end to end (the native conv kernels and MIOpen's igemm kernels are NHWC)
            self.model.to(memory_format=torch.channels_last)
        pdist.broadcast_module(self.model)
        self.params = [p for p in self.model.parameters() if p.requires_grad]
        self.amp_dtype = lc.get('amp_dtype')
        comm = getattr(torch, lc.comm_dtype) if lc.get('comm_dtype') else None
        # the two-phase backward (parallel/dp.py backward_phased): encoder parameters are phase 1, everything
        # downstream of the encoders' outputs (core LSTM, heads, critics, value encoder) phase 0
        enc = {id(p) for n, p in self.model.named_parameters() if n.startswith('encoder.')}
        phase_of = (lambda p: 1 if id(p) in enc else 0)
        self.model.phase_cut = self._phased()
        use_master = lc.get('master_weights', None)
        if use_master is None:
            use_master = self.device.type == 'cuda' and self.amp_dtype == 'bfloat16'
        self.master = None
        if use_master:
            self.master = MasterWeights(self.model, bucket_mb=lc.bucket_mb, comm_dtype=comm, phase_of=phase_of)
            self.reducer = self.master.reducer
            self.opt_params = self.master.opt_params
        else:
            self.reducer = GradientReducer(self.params, bucket_mb=lc.bucket_mb, comm_dtype=comm, phase_of=phase_of)
            self.opt_params = self.params
            if self.device.type == 'cuda':
                from ..ops.native import defer_verify
                self.reducer.grad_hook = defer_verify
        # fp32 step: the weights' derived forms built once per optimizer step (MasterWeights owns its own registry)
        self.derived = None
        if self.master is None and self.device.type == 'cuda' and \
                os.environ.get('APPLESTAR_DERIVED_WEIGHTS', '1') != '0':
            from ..ops.native import DerivedWeights
            self.derived = DerivedWeights()
            for p in self.params:
                p._derived_forms = self.derived
        self.grad_clip = build_grad_clip(lc.grad_clip)
        # the step's health gate lives in ONE device scalar: a captured update graph reads it by address
        self._gate = torch.ones((), dtype=torch.float32, device=self.device) if self.device.type == 'cuda' else None
        self.graph = None
        self.reset_optimizer()

    # ------------------------------------------------------------------ optimizer
    def _graph_requested(self) -> bool:
        return self.device.type == 'cuda' and bool(self.cfg.learner.get('graph_step', False))

    def reset_optimizer(self):
        """Fresh optimizer state (also used after a league reset)."""
        lc = self.cfg.learner
        self.optimizer = build_optimizer(self.opt_params, lc, betas=self.ADAM_BETAS, eps=self.ADAM_EPS,
                                         device=self.device)
        self.lr_scheduler = None            # the RL learner's LR is constant (rl_learner.py: MultiStepLR, no milestones)
        if lc.get('lr_scheduler') is not None:
            from ..utils.lr_scheduler import build_lr_scheduler
            self.lr_scheduler = build_lr_scheduler(self.optimizer, lc.lr_scheduler)
        # clip + Adam as two / three native launches (utils/fused_optim.py) on the GPU
        from ..utils.fused_optim import FusedClipAdam
        self.fused_opt = None
        if self.device.type == 'cuda' and FUSED_CLIP_ADAM and FusedClipAdam.supported(self.optimizer, self.grad_clip):
            segments = None
            if self.master is not None and self.grad_clip.clip_type == 'momentum_norm':
                segments = {self.master.master: self.master.segments()}    # per-layer norms, as in fp32
            self.fused_opt = FusedClipAdam(self.optimizer, self.grad_clip.threshold
                                           if self.grad_clip.clip_type not in ('none', 'momentum_norm') else None,
                                           clip=self.grad_clip, device_hparams=self._graph_requested(),
                                           segments=segments)
        if getattr(self, 'graph', None) is not None:
            self.graph.reset()

    def _graph_capable(self) -> bool:
        return self._graph_requested() and self.fused_opt is not None and \
            self.grad_clip.clip_type in GRAPH_SAFE_CLIPS

    def _make_graph(self, fwd_bwd):
        if not self._graph_capable():
            return None
        from ..runtime.step_graph import GraphedTrainStep
        if self.master is not None:
            self.master.defer_allreduce = True     # the all-reduce runs between the two graphs
        g = GraphedTrainStep(fwd_bwd, self._reduce, self._update, device=self.device)
        g.pre_replay = self.fused_opt.prepare      # step count / bias corrections: host work outside the graph
        return g

    # ------------------------------------------------------------------ backward / reduce / update
    def _phased(self) -> bool:
        """Two-phase backward with the downstream buckets' all-reduce issued between the phases: multi-rank
        (``learner.overlap_backward``, default on), or forced on one rank by APPLESTAR_PHASED_BACKWARD=1 (tests).
        Decided once (the model then cuts its forward graph at the encoders' outputs, ``Model._encode``); a
        forward that made the cut must be followed by the phased backward, which ``backward`` ensures: it runs
        the two phases exactly when the forward left (output, leaf) pairs."""
        forced = os.environ.get('APPLESTAR_PHASED_BACKWARD', '')
        if forced:
            return forced == '1'
        return pdist.get_world_size() > 1 and bool(self.cfg.learner.get('overlap_backward', True))

    def backward(self, loss: torch.Tensor):
        self.reducer.zero_grad(buffers=False)    # backward overwrites every slot (and zeroes unused ones)
        from ..ops import native
        boundary = getattr(self.model, 'encoder_boundary', None)
        self.model.encoder_boundary = None
        phased = bool(boundary)
        defer = self.device.type == 'cuda' and self.master is None     # fp32: heads' dW beside the LSTM backward
        if defer:
            native.defer_begin(self.device, loss, owner=self)
        try:
            join = (lambda: native.defer_end(self.device)) if defer else None
            if self.master is not None:
                self.master.backward(loss, boundary if phased else None)
            elif phased:
                self.reducer.backward_phased(loss, boundary, before_copy=join)
            else:
                self.reducer.backward(loss, before_copy=join)
        finally:
            if defer:
                native.defer_end(self.device)

    def _lstm_gate(self):
        """1.0 / 0.0 device scalar: the split LSTM exchange has not / has timed out (ops.native.lstm_exchange_ok)."""
        if self.device.type != 'cuda':
            return None
        from ..ops import native
        return native.lstm_exchange_ok(self.device)

    def _reduce(self):
        """Cross-rank gradient average and the step's health gate (MIN over ranks, issued with the buckets).
        Runs eagerly between the two graphs of a multi-rank graphed step, inside the single graph on one rank."""
        handle = None
        if self._gate is not None:
            self._gate.copy_(self._lstm_gate())
            if pdist.get_world_size() > 1:
                import torch.distributed as dist
                handle = dist.all_reduce(self._gate, op=dist.ReduceOp.MIN, async_op=True)
        if self.master is not None:
            self.master.synchronize()
        else:
            self.reducer.synchronize()
        if handle is not None:
            handle.wait()

    def _update(self) -> torch.Tensor:
        gate = self._gate
        if self.fused_opt is not None:
            if self.fused_opt.clip is None:
                self.grad_clip.step += 1
            norm = self.fused_opt.step(gate)
        else:
            norm = self.grad_clip.apply(self.opt_params, gate=gate)
            self.optimizer.step()
        if self.master is not None:
            self.master.after_step()
        elif self.derived is not None:
            self.derived.refresh()
        return norm

    # ------------------------------------------------------------------ diagnostics / state
    def nonfinite_grads(self):
        """Names of parameters whose current gradient has a NaN / Inf (debugging aid; syncs)."""
        bad = []
        if self.master is not None:
            views = self.master._master_grad_views()
            for p in self.master.reducer.params:
                g = views.get(p, p.grad)
                if g is not None and not bool(torch.isfinite(g).all()):
                    bad.append(self.master.names[p])
        else:
            for n, p in self.model.named_parameters():
                if p.grad is not None and not bool(torch.isfinite(p.grad).all()):
                    bad.append(n)
        return bad

    def model_state_dict(self):
        """fp32 model weights (the master copies when the compute weights are bf16)."""
        return self.master.state_dict() if self.master is not None else self.model.state_dict()

    def load_model_state_dict(self, sd):
        if self.master is not None:
            return self.master.load_state_dict(sd)
        res = self.model.load_state_dict(sd, strict=False)
        if self.derived is not None:
            self.derived.invalidate()
        return res

    def on_model_changed(self):
        """Call after editing model weights in place (e.g. a value-network reset)."""
        if self.master is not None:
            self.master.sync_from_model()
        elif self.derived is not None:
            self.derived.invalidate()

    def state_dict(self):
        return {'model': self.model_state_dict(), 'optimizer': self.optimizer.state_dict(),
                'last_iter': self.iter, 'grad_clip': self.grad_clip.state_dict()}

    def load_state_dict(self, sd, load_optimizer=True):
        self.load_model_state_dict(sd['model'])
        if load_optimizer and 'optimizer' in sd:
            self.optimizer.load_state_dict(sd['optimizer'])
        if 'grad_clip' in sd:
            self.grad_clip.load_state_dict(sd['grad_clip'])
        self.iter = int(sd.get('last_iter', 0))
        if self.graph is not None:
            self.graph.reset()

    def step_info(self, info: Dict) -> Dict:
        if self._gate is not None:
            info['lstm_exchange_ok'] = self._gate
        return info
