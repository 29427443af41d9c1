"""Host-side op switches (no GPU): the split-K switches are per host thread."""
import threading

from rdeic_amd import ops


def test_splitk_switch_is_thread_local():
    inside, release, seen = threading.Event(), threading.Event(), {}

    def other():
        with ops.splitk_allowed():
            inside.set()
            release.wait(10)
            seen["other_inside"] = ops.splitk_state()
        seen["other_after"] = ops.splitk_state()

    t = threading.Thread(target=other)
    t.start()
    inside.wait(10)
    assert ops.splitk_state() == (False, False)  # another thread's region does not leak here
    with ops.splitk_allowed(short_k=True):
        assert ops.splitk_state() == (True, True)
        release.set()
        t.join()
        assert ops.splitk_state() == (True, True)  # the other thread leaving does not reset ours
    assert ops.splitk_state() == (False, False)
    assert seen["other_inside"] == (True, False)
    assert seen["other_after"] == (False, False)
