"""Session.host_buffer views and the session's lifetime (CPU, fake library).

ADVICE r4: the arrays host_buffer returns point into the session's pinned
arena, which fdcn_session_destroy resets and the next session reuses.  A view
held past ``with Session()`` (a traceback keeping a plan alive) must not be
left pointing into recycled memory: the array owns an object that keeps the
session alive, and close() defers the destroy until the last view is gone.
The library is faked (no GPU here): these tests check the bookkeeping only.
"""
import gc

import numpy as np
import pytest

from finite_difference_amd import capi
from finite_difference_amd import session as sess


class _FakeLib:
    _fdcn_session_bound = True

    def __init__(self):
        self.arena = np.zeros(4096)
        self.destroyed = 0

    def fdcn_session_create(self, pref):
        pref._obj.value = 0x1000
        return 0

    def fdcn_session_destroy(self, h):
        self.destroyed += 1
        return 0

    def fdcn_session_host_buffer(self, h, nbytes, pref):
        assert nbytes <= self.arena.nbytes
        pref._obj.value = self.arena.ctypes.data
        return 0


@pytest.fixture
def fake(monkeypatch):
    L = _FakeLib()
    monkeypatch.setattr(capi, "lib", lambda: L)
    monkeypatch.setattr(capi, "require_device", lambda: None)
    return L


def test_view_defers_the_destroy_until_it_is_dropped(fake):
    S = sess.Session()
    a = S.host_buffer(10)
    assert a.shape == (10,) and a.dtype == np.float64
    a[:] = np.arange(10.0)
    assert fake.arena[3] == 3.0  # the view writes the pinned memory itself
    v = a[2:5].reshape(3, 1)
    del a
    S.close()
    assert fake.destroyed == 0 and S.close_pending and not S.closed
    with pytest.raises(capi.FdcnError):
        S.host_buffer(4)  # no new views of a session on its way out
    assert v[0, 0] == 2.0
    del v
    gc.collect()
    assert fake.destroyed == 1 and S.closed and not S.close_pending
    S.close()
    assert fake.destroyed == 1


def test_with_block_exit_on_an_exception_keeps_the_view_valid(fake):
    held = []
    with pytest.raises(RuntimeError):
        with sess.Session() as S:
            plan = S.host_buffer(8).reshape(2, 4)
            held.append(plan)  # what a traceback would keep alive
            raise RuntimeError("march failed")
    assert fake.destroyed == 0 and S.close_pending
    held.clear()
    del plan
    gc.collect()
    assert fake.destroyed == 1


def test_no_views_destroys_at_once(fake):
    with sess.Session() as S:
        b = S.host_buffer(3)
        del b
        gc.collect()
    assert fake.destroyed == 1 and S.closed


def test_views_keep_the_session_object_alive(fake):
    S = sess.Session()
    a = S.host_buffer(5)
    del S
    gc.collect()
    assert fake.destroyed == 0  # the view's owner holds the session
    owner = a.base
    while not isinstance(owner, sess._PinnedView):
        owner = owner.base
    assert owner.session.close_pending is False
    owner.session.close()
    del a, owner
    gc.collect()
    assert fake.destroyed == 1


def test_last_view_dropped_on_another_thread_leaves_destroy_pending(fake):
    """the session's device context goes back to the destroying
    thread's pool, so a deferred destroy runs on the creating thread only.
    The last view dropped on a worker thread leaves the session pending; the
    creating thread's next close() destroys it."""
    import threading
    S = sess.Session()
    box = [S.host_buffer(8)]
    S.close()
    assert S.close_pending and fake.destroyed == 0

    def drop():
        box.pop()
        gc.collect()
    t = threading.Thread(target=drop)
    t.start()
    t.join()
    assert not box
    gc.collect()
    assert fake.destroyed == 0 and S.close_pending and not S.closed
    S.close()  # the creating thread, no view left
    assert fake.destroyed == 1 and S.closed


def test_last_view_dropped_on_the_creating_thread_destroys(fake):
    S = sess.Session()
    a = S.host_buffer(8)
    S.close()
    del a
    gc.collect()
    assert fake.destroyed == 1 and S.closed
