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


def _bump(model, by):
    with torch.no_grad():
        for p in model.parameters():
            p.add_(by)


def test_subscriber_goes_stale_when_slot_is_replaced():
    """a subscriber mapped the old inode forever.  A slot unlinked and re-created (learner restart,
    reset_comm_setting) or re-created in place over a crashed learner's file (new session id) marks it stale."""
    a, b = _models('cpu')
    sd = a.policy_state_dict()
    name = _name('stale')
    pub = ModelPublisher(sd, shm_name=name)
    sub = ModelSubscriber(b, name, device='cpu')
    sub.bind(FlatLayout(sd))
    try:
        pub.publish(sd, last_iter=1)
        pub.wait()
        assert sub.poll() and not sub.stale
        pub.close(unlink=True)                       # a new inode at the same path
        _bump(a, 1.0)
        pub = ModelPublisher(a.policy_state_dict(), shm_name=name)
        pub.publish(a.policy_state_dict(), last_iter=2)
        pub.wait()
        assert not sub.poll() and sub.stale and not _check_equal(a, b)
        sub.close()
        sub = ModelSubscriber(b, name, device='cpu')  # re-attach: the new weights arrive
        sub.bind(FlatLayout(a.policy_state_dict()))
        assert sub.poll() and sub.last_iter == 2 and _check_equal(a, b)
        # a new publisher over the SAME file (crashed learner's slot left behind: O_CREAT on the existing inode)
        pub.slot.close(unlink=False)
        pub = ModelPublisher(a.policy_state_dict(), shm_name=name)
        assert not sub.poll() and sub.stale
    finally:
        sub.close()
        pub.close(unlink=True)


def test_subscriber_refuses_layout_with_equal_numel():
    """Layouts were compared by element count only: two tensors swapped keep the count but not the layout."""
    a, b = _models('cpu')
    sd = a.policy_state_dict()
    keys = list(sd)
    i = next(j for j in range(len(keys) - 1) if sd[keys[j]].numel() != sd[keys[j + 1]].numel())
    keys[i], keys[i + 1] = keys[i + 1], keys[i]
    swapped = {k: sd[k] for k in keys}
    name = _name('layout')
    pub = ModelPublisher(swapped, shm_name=name)
    sub = ModelSubscriber(b, name, device='cpu')
    try:
        with pytest.raises(ValueError):
            sub.bind(FlatLayout(sd))
    finally:
        sub.close()
        pub.close(unlink=True)


class _FakeAdapter:
    def __init__(self):
        self.msgs = []

    def pull(self, key, size=1, block=False):
        return [self.msgs.pop(0)] if self.msgs else []


def _actor_comm(server, adapter, experiment):
    from collections import deque
    from applestar_amd.actor.comm import ActorComm
    from applestar_amd.utils.config import AttrDict as Config
    comm = ActorComm.__new__(ActorComm)
    comm._cfg = Config({'common': {'experiment_name': experiment},
                        'actor': {'shared_model_slot': True, 'shared_model_slot_stale_s': 0.0}})
    comm._adapter, comm._interval, comm._last_update = adapter, 0.0, -1.0
    comm._last_reset, comm.update_times = {}, deque(maxlen=10)
    comm._attached, comm._attach_t, comm._slot_seen = {}, 0.0, {}
    comm.job = {'update_players': ['MP0']}
    return comm


def test_actor_reattaches_recreated_slot_and_falls_back_to_broadcast():
    """The actor picks up a re-created slot's weights, and takes the network broadcast when the slot stops
    advancing behind it (stale slot of a dead learner)."""
    from applestar_amd.actor.inference import InferenceServer
    from applestar_amd.learner.rl_learner import model_slot_name
    a, b = _models('cpu')
    srv = InferenceServer(device='cpu', amp_dtype=None)
    srv.set_model('MP0', b)
    exp = f'exp{os.getpid()}'
    name = model_slot_name('MP0', exp)
    assert exp in name and model_slot_name('MP0', 'other') != name
    pub = ModelPublisher(a.policy_state_dict(), shm_name=name)
    adapter = _FakeAdapter()
    comm = _actor_comm(srv, adapter, exp)

    class _Actor:
        _server = srv

        def reset_env(self):
            pass
    try:
        pub.publish(a.policy_state_dict(), last_iter=3)
        pub.wait()
        comm.update_model(_Actor())
        assert comm._attached['MP0'] and srv.model_iter['MP0'] == 3 and _check_equal(a, b)
        # learner restarts: slot unlinked and re-created with new weights
        pub.close(unlink=True)
        _bump(a, 0.5)
        pub = ModelPublisher(a.policy_state_dict(), shm_name=name)
        pub.publish(a.policy_state_dict(), last_iter=4)
        pub.wait()
        comm.update_model(_Actor())                  # sees 'stale', detaches
        comm.update_model(_Actor())                  # re-attaches, loads the new slot
        assert srv.model_iter['MP0'] == 4 and _check_equal(a, b)
        # the slot stops advancing while the broadcast moves on: the newer broadcast wins and the slot is dropped
        _bump(a, 0.25)
        net = ModelPublisher(a.policy_state_dict())
        net.publish(a.policy_state_dict(), last_iter=9)
        adapter.msgs.append(net.payload())
        comm.update_model(_Actor())
        assert srv.model_iter['MP0'] == 9 and _check_equal(a, b) and srv.model_slot_state('MP0') is None
    finally:
        srv.detach_model_slot('MP0')
        pub.close(unlink=True)


def test_slot_of_exited_learner_is_not_attached(tmp_path):
    """A slot a terminated learner left in /dev/shm (no unlink) still holds that run's last weights: the next
    run's inference server must not attach it (the publisher's pid is in the header)."""
    import subprocess
    import sys
    from applestar_amd.actor.inference import InferenceServer
    name = _name('dead')
    code = ("import os, sys, torch; sys.path.insert(0, %r)\n"
            "from applestar_amd.models.model import Model\n"
            "from applestar_amd.runtime.flat_model import ModelPublisher\n"
            "m = Model({}); sd = m.policy_state_dict(); p = ModelPublisher(sd, shm_name=%r)\n"
            "p.publish(sd, last_iter=7); p.wait(); os._exit(0)\n") % (os.path.dirname(os.path.dirname(
                os.path.abspath(__file__))), name)
    subprocess.run([sys.executable, '-c', code], check=True, timeout=300)
    try:
        assert os.path.exists('/dev/shm/' + name)
        _, b = _models('cpu')
        srv = InferenceServer(device='cpu', amp_dtype=None)
        srv.set_model('MP0', b)
        assert not srv.attach_model_slot('MP0', name) and srv.model_slot_state('MP0') is None
    finally:
        os.unlink('/dev/shm/' + name)
