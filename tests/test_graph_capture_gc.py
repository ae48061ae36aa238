"""HIP-graph capture helpers that need no GPU (runtime/graphs.py).

``gc_paused`` keeps Python's cyclic collector off for the duration of a capture (a collection mid-capture aborted the
graphed train step, profiles/r10zk_*): it must collect first, pause, and restore the previous state - also when the
captured body raises, and without re-enabling a collector the caller had disabled."""
import gc

import pytest

from applestar_amd.runtime.graphs import gc_paused


def test_gc_paused_disables_and_restores():
    assert gc.isenabled()
    with gc_paused():
        assert not gc.isenabled()
    assert gc.isenabled()


def test_gc_paused_restores_after_exception():
    with pytest.raises(RuntimeError):
        with gc_paused():
            raise RuntimeError('capture failed')
    assert gc.isenabled()


def test_gc_paused_keeps_a_disabled_collector_disabled():
    gc.disable()
    try:
        with gc_paused():
            assert not gc.isenabled()
        assert not gc.isenabled()
    finally:
        gc.enable()


def test_gc_paused_collects_pending_cycles_first():
    class Node:
        pass

    a, b = Node(), Node()
    a.other, b.other = b, a
    import weakref
    ref = weakref.ref(a)
    del a, b
    with gc_paused():
        assert ref() is None
