"""Micro-batcher failure handling: fallback re-run, quarantine, CPU takeover,
watchdog, gpu_fail fault injection — all with CPU fake runners."""
import numpy as np
import pytest

from routest_amd.models.features import pack_record
from routest_amd.serve.batcher import MicroBatcher
from routest_amd.utils.faults import clear_faults, maybe_fail, set_faults
from routest_amd.utils.metrics import REGISTRY
from routest_amd.utils.timeutil import parse_iso


def _rec(d=5000.0):
    return pack_record(weather="Sunny", traffic="Low", distance_m=d,
                       pickup=parse_iso("2025-08-25T08:30:00"), driver_age=30)


class FlakyRunner:
    def __init__(self, fail_first):
        self.fail_first, self.calls = fail_first, 0

    def __repr__(self):
        return "FlakyRunner"

    def __call__(self, rec):
        self.calls += 1
        if self.calls <= self.fail_first:
            raise RuntimeError("device lost")
        return np.full(len(rec), 7.0, np.float32)


def cpu_runner(rec):
    return np.full(len(rec), 3.0, np.float32)


def test_failed_batch_rerun_on_fallback():
    b = MicroBatcher([FlakyRunner(1)], batch_max=8, timeout_us=0, fallback=cpu_runner)
    try:
        assert b.predict_sync(_rec()) == 3.0      # failed on the device, served by the fallback
        assert b.predict_sync(_rec()) == 7.0      # device recovered
        assert not b.degraded
    finally:
        b.close()


def test_quarantine_then_cpu_takeover():
    f0 = REGISTRY.device_failures.value()
    b = MicroBatcher([FlakyRunner(10 ** 9)], batch_max=8, timeout_us=0, fallback=cpu_runner, max_failures=2)
    try:
        vals = [b.predict_sync(_rec(), timeout=10) for _ in range(6)]
        assert vals == [3.0] * 6
        assert b.degraded
        h = b.health()
        assert h[0]["healthy"] is False and h[-1]["runner"] == "cpu-fallback"
        assert REGISTRY.device_failures.value() - f0 == 2   # quarantined after 2, then CPU worker
    finally:
        b.close()


def test_without_fallback_errors_propagate():
    b = MicroBatcher([FlakyRunner(1)], batch_max=8, timeout_us=0)
    try:
        with pytest.raises(RuntimeError):
            b.predict_sync(_rec(), timeout=10)
        assert b.predict_sync(_rec(), timeout=10) == 7.0
    finally:
        b.close()


def test_watchdog_counts_slow_batches():
    import time

    def slow(rec):
        time.sleep(0.02)
        return np.zeros(len(rec), np.float32)
    s0 = REGISTRY.slow_batches.value()
    b = MicroBatcher([slow], batch_max=8, timeout_us=0, watchdog_ms=5)
    try:
        b.predict_sync(_rec())
        assert REGISTRY.slow_batches.value() - s0 >= 1
    finally:
        b.close()


def test_gpu_fail_fault_injection():
    set_faults("gpu_fail")
    try:
        with pytest.raises(Exception):
            maybe_fail("gpu_fail")
    finally:
        clear_faults()
    maybe_fail("gpu_fail")  # cleared


def test_service_reports_runner_health():
    from routest_amd.models.mlp3 import LinearETA
    from routest_amd.serve.eta_service import EtaService
    from routest_amd.data.synth import synth_trips
    x, y = synth_trips(500, 0)
    svc = EtaService(model=LinearETA().fit(x, y), device="cpu")
    try:
        d = svc.describe()
        assert "runners" in d and d["degraded"] is False
    finally:
        svc.close()


def test_inline_when_idle_and_queue_under_load():
    import asyncio
    calls = []

    def runner(rec):
        calls.append(len(rec))
        return np.full(len(rec), 2.0, np.float32)
    b = MicroBatcher([runner], batch_max=64, timeout_us=2000)
    try:
        async def one():
            return await b.submit(_rec())
        assert asyncio.run(one()) == 2.0 and calls == [1]

        async def many():
            b._busy += 1          # pretend a batch is in flight: everything must queue
            try:
                return await asyncio.gather(*[b.submit(_rec()) for _ in range(32)])
            finally:
                b._busy -= 1
        assert asyncio.run(many()) == [2.0] * 32
        assert sum(calls[1:]) == 32
    finally:
        b.close()


def test_two_consumers_never_strand_requests():
    """Two workers on one queue, bursts of concurrent requests: every request is answered.  With
    CPython's timed SimpleQueue.get a worker whose wake-up item was taken by the other worker
    re-waited without a timeout and held its partial batch until the next put (utils/queues.py);
    this lost requests within ~10 bursts."""
    import concurrent.futures as cf
    import time

    from routest_amd.data.synth import synth_records

    import threading
    lock = threading.Lock()

    class Slow:
        rows = 0

        def __call__(self, rec):
            time.sleep(0.0002)
            with lock:                      # (two workers: a bare += can lose an update)
                Slow.rows += len(rec)
            return np.arange(len(rec), dtype=np.float32)

    rec, _ = synth_records(6000, 1)
    for _ in range(20):
        Slow.rows = 0
        mb = MicroBatcher([Slow(), Slow()], batch_max=512, timeout_us=300, inline_when_idle=False)
        try:
            with cf.ThreadPoolExecutor(16) as ex:
                futs = [ex.submit(mb.predict_sync, rec[i].item(), 5.0) for i in range(len(rec))]
                for f in futs:
                    f.result(10)
        finally:
            mb.close()
        assert Slow.rows == len(rec)


def test_get_until_deadline():
    import queue
    import time

    from routest_amd.utils.queues import get_until
    q = queue.SimpleQueue()
    t0 = time.perf_counter()
    with pytest.raises(queue.Empty):
        get_until(q, t0 + 0.002)
    assert time.perf_counter() - t0 < 0.5
    q.put(7)
    assert get_until(q, time.perf_counter() + 1.0) == 7
