"""CPU: the frame engine's failure handling without a device (csrc/engine.cpp FrameEngine::Pool,
srtEnginePoolSelfTest).

One worker throws, or stalls, while every other worker waits for a release that only the abort gives
-- as engine workers wait in RCCL on a peer that will never send. The run must end with the first
error within the deadline, with the abort hook (ncclCommAbort on every communicator, in the engine)
run exactly once: the reference's convention is an error status plus a message, never a hang
(model_runner/context.cpp:40-48).
"""
from __future__ import annotations

import pytest

from simpleraytracer_amd.engine import pool_self_test


@pytest.mark.parametrize("workers,failing", [(1, 0), (2, 1), (8, 3)])
def test_pool_worker_failure_aborts_the_others(workers, failing):
    msg, elapsed, calls = pool_self_test(workers, failing, "fail", timeout_s=5.0)
    assert msg == f"injected failure of worker {failing}"
    assert calls == 1
    assert elapsed < 2.0  # the failure itself triggers the abort: no deadline involved


@pytest.mark.parametrize("workers,failing", [(1, 0), (4, 2)])
def test_pool_stall_hits_the_deadline(workers, failing):
    msg, elapsed, calls = pool_self_test(workers, failing, "stall", timeout_s=0.5)
    assert "no device made progress" in msg
    assert calls == 1
    assert 0.5 <= elapsed < 5.0


def test_pool_self_test_rejects_bad_arguments():
    from simpleraytracer_amd.device import SrtError

    with pytest.raises(SrtError, match="Bad argument"):
        pool_self_test(2, 2, "fail")
