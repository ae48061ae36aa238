"""Learner -> actor model hand-off as one flat snapshot with a version counter (runtime/flat_model.py,
VERDICT r4 weak 7: replaces ~430 per-tensor D2H copies + clone + TCP)."""
import os

import pytest
import torch

from applestar_amd.models.model import Model
from applestar_amd.runtime.flat_model import FlatLayout, ModelPublisher, ModelSubscriber


def _name(tag):
    return f'applestar_test_{tag}_{os.getpid()}'


def _models(device):
    torch.manual_seed(0)
    a = Model({}).to(device)
    torch.manual_seed(1)
    b = Model({}).to(device)
    return a, b


def _check_equal(a, b):
    sa, sb = a.policy_state_dict(), b.state_dict()
    return all(torch.equal(sb[k], v) for k, v in sa.items())


def _roundtrip(device):
    a, b = _models(device)
    sd = a.policy_state_dict()
    pub = ModelPublisher(sd, shm_name=_name('rt'))
    sub = ModelSubscriber(b, _name('rt'), device=device)
    try:
        sub.bind(FlatLayout(sd))
        assert not sub.poll() and not _check_equal(a, b)
        pub.publish(sd, last_iter=11)
        pub.wait()
        assert sub.poll() and sub.last_iter == 11 and _check_equal(a, b)
        assert not sub.poll()                                   # same version: nothing to do
        with torch.no_grad():
            for p in a.parameters():
                p.add_(1.0)
        pub.publish(a.policy_state_dict(), last_iter=12, reset_flag=True)
        assert pub.slot.read_header()[0] % 2 == 1              # in flight: readers skip it
        assert not sub.poll()
        pub.wait()
        assert sub.poll() and sub.reset_flag and _check_equal(a, b)
        # the cross-host message: one flat tensor + layout
        msg = pub.payload()
        assert set(msg) == {'flat_model', 'names', 'shapes', 'model_last_iter', 'reset_flag'}
        assert msg['flat_model'].numel() == pub.layout.numel
    finally:
        sub.close()
        pub.close(unlink=True)
    assert not os.path.exists('/dev/shm/' + _name('rt'))


def test_flat_model_roundtrip_cpu():
    _roundtrip('cpu')


def test_inference_server_load_flat_cpu():
    from applestar_amd.actor.inference import InferenceServer
    a, b = _models('cpu')
    srv = InferenceServer(device='cpu', amp_dtype=None)
    srv.set_model("MP0", b)
    pub = ModelPublisher(a.policy_state_dict())
    pub.publish(a.policy_state_dict(), last_iter=5)
    msg = pub.payload()
    srv.load_flat('MP0', msg['flat_model'], msg['names'], msg['shapes'], last_iter=msg['model_last_iter'])
    assert _check_equal(a, b) and srv.model_iter['MP0'] == 5


@pytest.mark.gpu
def test_flat_model_roundtrip_gpu():
    """On the GPU: pinned (hipHostRegister'ed) /dev/shm slot, one D2H / H2D DMA each way, native multi-copies;
    channels_last conv weights round-trip by value."""
    _roundtrip(torch.device('cuda', 0))
