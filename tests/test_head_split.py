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
