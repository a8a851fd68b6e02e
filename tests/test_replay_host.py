"""Host logic of the recorded-step replay (autoformer_amd/replay.py) on CPU: calls are re-issued in
order with their recorded arguments, ctypes structures are frozen at record time, a non-zero return
raises, markers run in place."""
import ctypes

import pytest

from autoformer_amd import replay as R


class _S(ctypes.Structure):
    _fields_ = [("a", ctypes.c_int), ("p", ctypes.c_void_p)]


def test_replay_reissues_calls_in_order_with_frozen_structs():
    log = []
    rec = R.StepRecord()
    s = _S(1, 0x1000)
    rec.add_native(lambda st, n: log.append(("f", st.a, st.p, n)) or 0, "f", (s, 7))
    s.a = 99  # the caller reuses its descriptor object after the call
    rec.add_marker(lambda: log.append("marker"))
    rec.add_native(lambda n: log.append(("g", n)) or 0, "g", (3,))
    rec.replay()
    rec.replay()
    assert log == [("f", 1, 0x1000, 7), "marker", ("g", 3)] * 2
    assert rec.native_calls() == 2


def test_replay_raises_on_library_error(monkeypatch):
    from autoformer_amd import _lib as L

    seen = []
    monkeypatch.setattr(L, "check", lambda rc, what="": seen.append((rc, what)) or (_ for _ in ()).throw(
        RuntimeError(f"{what} failed ({rc})")))
    rec = R.StepRecord()
    rec.add_native(lambda: 5, "avc_broken", ())
    with pytest.raises(RuntimeError, match="avc_broken failed"):
        rec.replay()
    assert seen == [(5, "avc_broken")]


def test_recording_hook_is_off_outside_a_recording():
    from autoformer_amd import _lib as L

    assert L._REC is None
