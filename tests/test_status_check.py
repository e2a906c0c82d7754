"""The opt-in device status check's host logic (CPU): only the outermost of nested
status-checked calls reads the words, only the devices its launches touched are read, nothing is
read during CUDA graph capture or with the check off.  (The GPU side -- a flagged word raising
and being cleared -- is tests/test_device_status.py.)"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))

from kvcompress import _engine as E  # noqa: E402


@pytest.fixture
def reads(monkeypatch):
    got = []
    monkeypatch.setattr(E, "raise_on_status", lambda devices=None: got.append(set(devices)))
    monkeypatch.setattr(E.torch.cuda, "is_current_stream_capturing", lambda: False)
    prev = E.set_status_check(True)
    yield got
    E.set_status_check(prev)


def _launch(device):
    """What status_word() records for a launch on `device` (without making the word)."""
    t = E._check_state.touched
    if t is not None:
        t.add(device)


@E.status_checked
def _inner(device):
    _launch(device)
    return device


@E.status_checked
def _outer():
    _launch(5)
    return [_inner(3), _inner(3)]


def test_nested_checked_calls_read_once_at_the_outermost(reads):
    assert _outer() == [3, 3]
    assert reads == [{3, 5}]
    assert _inner(2) == 2  # a top-level call reads on its own
    assert reads == [{3, 5}, {2}]


def test_no_read_without_launches_or_with_the_check_off(reads):
    @E.status_checked
    def idle():
        return 0
    idle()
    assert reads == []
    E.set_status_check(False)
    _outer()
    assert reads == []


def test_no_read_while_capturing(reads, monkeypatch):
    monkeypatch.setattr(E.torch.cuda, "is_current_stream_capturing", lambda: True)
    _outer()
    assert reads == []


def test_state_reset_after_an_exception(reads):
    @E.status_checked
    def boom():
        _launch(1)
        raise ValueError("x")
    with pytest.raises(ValueError):
        boom()
    assert reads == []
    assert E._check_state.depth == 0 and E._check_state.touched is None
    _inner(4)
    assert reads == [{4}]


def test_output_devices_of_a_result():
    """The native replay bypasses status_word(): the memo wrapper reads the devices of the
    result's CUDA tensors (none for CPU tensors or a non-list result)."""
    import torch
    t = torch.zeros(1)
    assert E._output_devices([(t, t)]) == set()
    assert E._output_devices(None) == set()
