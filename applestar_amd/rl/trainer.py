"""One RL learner iteration (forward -> loss -> backward -> all-reduce -> clip -> Adam).

Step semantics of ``RLLearner._train`` (``distar/agent/default/rl_learner.py:82-145``): Adam with
betas (0, 0.99), eps 1e-5, ``pytorch_norm`` clip at 1.0, value pre-training phase that trains only
the critic for ``value_pretrain_iters`` iterations.  MI355X specifics: bf16 autocast for every GEMM /
conv (fp32 master weights, fp32 LayerNorm/softmax/loss), gradients all-reduced in overlapped buckets
over RCCL, sync-free logging.
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, Optional

import torch

from ..utils.optim import build_optimizer
from ..models.model import Model
from ..parallel import dist as pdist
from ..parallel.dp import GradientReducer
from ..parallel.mixed import MasterWeights
from ..utils.config import AttrDict, deep_merge_dicts
from ..utils.grad_clip import build_grad_clip
from .loss import ReinforcementLoss

DEFAULT_LEARNER_CONFIG = AttrDict({
    'learner': {
        'player_id': 'MP0',
        'learning_rate': 1e-5,
        'weight_decay': 0.0,
        'use_value_feature': True,
        'value_pretrain_iters': -1,
        'grad_clip': {'type': 'pytorch_norm', 'threshold': 1.0},
        'bucket_mb': 32,
        'comm_dtype': None,
        'amp_dtype': 'bfloat16',
        # HIP-graph capture of the whole step (runtime/step_graph.py); GPU only.  Off by default: a replay
        # issues in ~1.5 ms of host time, but the captured step runs 29.8 vs 27.3 ms on the GPU (bf16,
        # profiles/r3l_graph_sync_probe.txt) - it pays only when the host, not the GPU, is the bottleneck
        'graph_step': False,
    },
    'model': {'enable_baselines': ['winloss']},
})


def _amp(device: torch.device, dtype_name: Optional[str]):
    if device.type != 'cuda' or not dtype_name:
        return contextlib.nullcontext()
    # no autocast weight cache: the compute weights are already bf16 (master weights), and a cache
    # must not outlive a HIP-graph capture
    return torch.autocast('cuda', dtype=getattr(torch, dtype_name), cache_enabled=False)


FUSED_CLIP_ADAM = os.environ.get('APPLESTAR_FUSED_ADAM', '1') != '0'     # A/B switch

# grad-clip types whose state is all on the device (safe to replay from a graph)
_GRAPH_SAFE_CLIPS = ('none', 'pytorch_norm', 'clip_norm', 'clip_const')


class RLTrainer:
    def __init__(self, cfg: Optional[dict] = None, device='cpu', model: Optional[Model] = None):
        self.cfg = deep_merge_dicts(DEFAULT_LEARNER_CONFIG, cfg or {})
        lc = self.cfg.learner
        self.device = torch.device(device)
        self.model = model if model is not None else Model(self.cfg, use_value_network=True)
        self.model.to(self.device)
        if self.device.type == 'cuda':
            # MIOpen find-mode autotuning (cudnn.benchmark) is opt-in: it measured ~10% faster convs on the
            # bench shapes, but two runs that used it left the GPU in a memory-fault state
            torch.backends.cudnn.benchmark = bool(lc.get('conv_autotune', False))
            # NHWC convolutions end to end (MIOpen igemm kernels are NHWC)
            self.model.to(memory_format=torch.channels_last)
        pdist.broadcast_module(self.model)
        self.params = [p for p in self.model.parameters() if p.requires_grad]
        comm = getattr(torch, lc.comm_dtype) if lc.get('comm_dtype') else None
        use_master = lc.get('master_weights', None)
        if use_master is None:
            use_master = self.device.type == 'cuda' and lc.get('amp_dtype') == 'bfloat16'
        self.master = None
        if use_master:
            self.master = MasterWeights(self.model, bucket_mb=lc.bucket_mb, comm_dtype=comm)
            self.reducer = self.master.reducer
            self.opt_params = self.master.opt_params
        else:
            self.reducer = GradientReducer(self.params, bucket_mb=lc.bucket_mb, comm_dtype=comm)
            self.opt_params = self.params
        # fp32 step: the weights' derived forms (transposed GEMM weights, flipped conv weights) rebuilt once per
        # optimizer step in a few multi-tensor launches instead of one transpose / flip copy per layer and call
        self.derived = None
        if self.master is None and self.device.type == 'cuda' and not lc.get('graph_step', False):
            from ..ops.native import DerivedWeights
            self.derived = DerivedWeights()
            for p in self.params:
                p._derived_forms = self.derived
        self.grad_clip = build_grad_clip(lc.grad_clip)
        self.reset_optimizer()
        self.loss = ReinforcementLoss(lc, lc.player_id)
        self.iter = 0
        self.remain_value_pretrain = int(lc.get('value_pretrain_iters', -1))
        self.amp_dtype = lc.get('amp_dtype')
        self.graph = None
        if self._graph_capable():
            from ..runtime.step_graph import GraphedTrainStep
            if self.master is not None:
                self.master.defer_allreduce = True     # the all-reduce runs between the two graphs
            self.graph = GraphedTrainStep(self._fwd_bwd, self._reduce, self._update, device=self.device)
            if self.master is not None and self.master.derived is not None:
                self.master.derived.enabled = False    # per-call forms inside the captured step

    def _graph_capable(self) -> bool:
        lc = self.cfg.learner
        return (self.device.type == 'cuda' and bool(lc.get('graph_step', False)) and self.master is not None and
                self.grad_clip.clip_type in _GRAPH_SAFE_CLIPS and isinstance(self.optimizer, torch.optim.Adam) and
                self.optimizer.defaults.get('capturable', False))

    def reset_optimizer(self):
        """Fresh Adam(betas=(0, 0.99), eps=1e-5) state (also used after a league reset)."""
        lc = self.cfg.learner
        capturable = self.device.type == 'cuda' and bool(lc.get('graph_step', False))
        self.optimizer = build_optimizer(self.opt_params, lc, betas=(0.0, 0.99), eps=1e-5, device=self.device,
                                         capturable=capturable)
        self.lr_scheduler = None
        # clip + Adam as two native launches (utils/fused_optim.py) on the eager GPU step; the graph-captured step
        # keeps torch's capturable Adam (its bias corrections are host floats here)
        from ..utils.fused_optim import FusedClipAdam
        self.fused_opt = None
        if self.device.type == 'cuda' and not capturable and FUSED_CLIP_ADAM and \
                FusedClipAdam.supported(self.optimizer, self.grad_clip):
            self.fused_opt = FusedClipAdam(self.optimizer, self.grad_clip.threshold
                                           if self.grad_clip.clip_type != 'none' else None)
        if getattr(self, 'graph', None) is not None:
            self.graph.reset()

    def _value_pretrain_toggle(self):
        active = self.remain_value_pretrain > 0
        self.model.only_update_baseline = active
        self.loss.only_update_value = active
        if active:
            self.remain_value_pretrain -= 1

    # ------------------------------------------------------------------ one iteration, in three parts
    def _fwd_bwd(self, batch: Dict) -> Dict[str, torch.Tensor]:
        if not self.model.training:   # train() walks ~670 modules: ~1 ms of host time per step
            self.model.train()
        with _amp(self.device, self.amp_dtype):
            out = self.model.rl_learner_forward(**batch)
        info = self.loss.compute_loss(out)
        self.reducer.zero_grad(buffers=False)    # backward overwrites every slot (and zeroes unused ones)
        if self.master is not None:
            self.master.backward(info['total_loss'])
        else:
            self.reducer.backward(info['total_loss'])
        # detached: a returned loss must not keep this step's autograd graph (and its AccumulateGrad nodes,
        # bound to the stream they were created on) alive into the next step - or into a graph capture
        return {k: (v.detach() if torch.is_tensor(v) else v) for k, v in info.items()}

    def _reduce(self):
        if self.master is not None:
            self.master.synchronize()
        else:
            self.reducer.synchronize()

    def _update(self) -> torch.Tensor:
        gate = self._lstm_gate()
        if self.fused_opt is not None:
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

    def _lstm_gate(self):
        """1.0 / 0.0 device scalar: the split LSTM exchange has not / has timed out (ops.native.lstm_exchange_ok);
        logged with the step's scalars as ``lstm_exchange_ok`` (the learner raises on 0)."""
        if self.device.type != 'cuda':
            return None
        from ..ops import native
        self._gate = native.lstm_exchange_ok(self.device)
        return self._gate

    def step(self, batch: Dict) -> Dict[str, torch.Tensor]:
        self._value_pretrain_toggle()
        if self.graph is not None and 'entity_total' in batch:
            from ..models.encoders import entity_pad_for
            b = dict(batch)
            total = b.pop('entity_total')
            b['entity_pad'] = entity_pad_for(total, b['entity_info']['unit_type'].shape[1])
            info = self.graph(b, extra_key=(self.model.only_update_baseline,))
        else:
            info = self._fwd_bwd(batch)
            self._reduce()
            info['gradient'] = self._update()
            if getattr(self, '_gate', None) is not None:
                info['lstm_exchange_ok'] = self._gate
        self.iter += 1
        return info

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
        return self.model.load_state_dict(sd, strict=False)

    def on_model_changed(self):
        """Call after editing model weights in place (e.g. a value-network reset)."""
        if self.master is not None:
            self.master.sync_from_model()

    def state_dict(self):
        return {'model': self.model_state_dict(), 'optimizer': self.optimizer.state_dict(),
                'last_iter': self.iter, 'grad_clip': self.grad_clip.state_dict()}

    def load_state_dict(self, sd, load_optimizer=True):
        self.load_model_state_dict(sd['model'])
        if load_optimizer and 'optimizer' in sd:
            self.optimizer.load_state_dict(sd['optimizer'])
        self.iter = int(sd.get('last_iter', 0))
