"""The teacher-forced head splits used by ``Policy.train_forward``'s side-stream path (models/heads.py), on the CPU:
each split must reproduce the unsplit head exactly enough that only the stream placement differs.

* action-type / delay / queued: ``teacher_logits`` + ``teacher_embedding`` == the head's teacher-forced forward;
* selected units: ``forward_teacher(split=True)`` + ``pointer_logits`` == ``forward_teacher`` (logits and the
  output embedding), for every entity-reduce type."""
import pytest
import torch

from applestar_amd.models import heads


def _close(a, b, tol=2e-6):
    return float((a - b).abs().max()) <= tol * max(1.0, float(b.abs().max()))


def test_action_type_split_matches_forward():
    torch.manual_seed(0)
    h = heads.ActionTypeHead()
    lstm, ctx = torch.randn(6, 384), torch.randn(6, 448)
    at = torch.randint(0, h.action_num, (6,))
    logits, _, emb = h(lstm, ctx, 0.8, action_type=at)
    assert _close(h.teacher_logits(lstm, ctx, 0.8), logits)
    assert _close(h.teacher_embedding(lstm, ctx, at), emb)


@pytest.mark.parametrize('cls', [heads.DelayHead, heads.QueuedHead])
def test_arg_head_split_matches_forward(cls):
    torch.manual_seed(1)
    h = cls()
    e = torch.randn(6, 1024)
    a = torch.randint(0, h.n_out, (6,))
    logits, _, emb = h(e, 0.7, action=a)
    assert _close(h.teacher_logits(e, 0.7), logits)
    assert _close(h.teacher_embedding(e, a), emb)


@pytest.mark.parametrize('reduce_type', heads.SelectedUnitsHead.REDUCE_TYPES)
def test_selected_units_split_matches_forward_teacher(reduce_type):
    torch.manual_seed(2)
    su = heads.SelectedUnitsHead(reduce_type=reduce_type)
    B, N = 5, 30
    ae0, ee = torch.randn(B, 1024), torch.randn(B, N, 256)
    en = torch.tensor([1, 7, 30, 12, 3])
    sun = torch.tensor([0, 3, 64, 5, 1])
    sel = torch.randint(0, N, (B, 64))
    sel[torch.arange(B), sun.clamp(max=63)] = en        # end token after the selected units
    logits, _, emb, _ = su.forward_teacher(ae0, ee, en, sun, sel)
    ptr, emb2, _ = su.forward_teacher(ae0, ee, en, sun, sel, split=True)
    assert _close(emb2, emb, 1e-5)
    assert _close(su.pointer_logits(ptr), logits, 1e-5)


def test_selected_units_folded_queries_gradients_match():
    """The split pointer half takes query_fc1 folded into embed_fc2 (SU_FOLD): the loss gradients of every head
    parameter and of the input embedding match the unsplit (unfolded) head's."""
    torch.manual_seed(3)
    su = heads.SelectedUnitsHead()
    B, N = 4, 20
    ae0, ee = torch.randn(B, 1024), torch.randn(B, N, 256)
    en = torch.tensor([3, 20, 9, 1])
    sun = torch.tensor([2, 64, 4, 0])
    sel = torch.randint(0, N, (B, 64))
    sel[torch.arange(B), sun.clamp(max=63)] = en
    grads = []
    for split in (False, True):
        su.zero_grad()
        a = ae0.clone().requires_grad_()
        if split:
            ptr, emb, _ = su.forward_teacher(a, ee, en, sun, sel, split=True)
            logits = su.pointer_logits(ptr)
        else:
            logits, _, emb, _ = su.forward_teacher(a, ee, en, sun, sel)
        w = torch.linspace(-1, 1, logits.shape[-1])
        (torch.where(logits > -1e8, logits, 0) * w).sum().backward(retain_graph=True)
        (emb * emb).mean().backward()
        grads.append([a.grad.clone()] + [p.grad.clone() if p.grad is not None else torch.zeros_like(p)
                                         for p in su.parameters()])
    for g0, g1 in zip(*grads):
        assert _close(g1, g0, 2e-5), float((g1 - g0).abs().max())
