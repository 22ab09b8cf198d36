"""Stress the 2-runner MicroBatcher on one GPU (the configuration of
tests/test_multirank_gpu.py::test_micro_batcher_two_runners_same_answers, which once timed out):
N rounds of 6000 concurrent single-record requests; prints per-round time and the resident-scorer
stats.  Exits non-zero on any mismatch or request timeout."""
import concurrent.futures as cf
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from routest_amd.data.synth import synth_records, synth_trips  # noqa: E402
from routest_amd.models.mlp3 import EtaMLP  # noqa: E402
from routest_amd.ops.eta_mlp import EtaMlpKernel, records_to_tensor  # noqa: E402
from routest_amd.serve.batcher import GpuRunner, MicroBatcher  # noqa: E402


class Timed:
    """Runner proxy recording (start, seconds, rows, path) of every call."""

    def __init__(self, r, log):
        self.r, self.log = r, log
        self.resident = r.resident

    def __call__(self, rec):
        t0 = time.perf_counter()
        st0 = self.r.resident.stats() if self.r.resident is not None else None
        try:
            return self.r(rec)
        finally:
            st1 = self.r.resident.stats() if self.r.resident is not None else None
            self.log.append((t0, time.perf_counter() - t0, len(rec), repr(self.r), st0, st1))

    def close(self):
        self.r.close()

    def __repr__(self):
        return repr(self.r)


def main(rounds: int = 5) -> int:
    torch.manual_seed(0)
    m = EtaMLP(256)
    xs, ys = synth_trips(16384, 5)
    m.fit_normalization(xs, ys)
    dev = torch.device("cuda:0")
    k = EtaMlpKernel(m, dev)
    rc = 0
    for it in range(rounds):
        calls = []
        runners = [Timed(GpuRunner(k, dev, 512), calls), Timed(GpuRunner(k, dev, 512), calls)]
        mb = MicroBatcher(runners, batch_max=512, timeout_us=300, inline_when_idle=False)
        t0 = time.perf_counter()
        try:
            rec, _ = synth_records(6000, 31 + it)
            ref = k(records_to_tensor(rec).to(dev)).cpu().numpy()
            with cf.ThreadPoolExecutor(16) as ex:
                futs = [ex.submit(mb.predict_sync, rec[i].item(), 20.0) for i in range(len(rec))]
                got = np.array([f.result(40) for f in futs], dtype=np.float32)
            ok = np.array_equal(got, ref)
            st = runners[0].resident.stats() if runners[0].resident is not None else {}
            print(f"round {it}: {time.perf_counter() - t0:.2f} s equal={ok} resident={st}", flush=True)
            rc |= 0 if ok else 1
        except Exception as e:  # noqa: BLE001
            print(f"round {it}: FAILED after {time.perf_counter() - t0:.1f} s: {e!r}", flush=True)
            import faulthandler
            faulthandler.dump_traceback(all_threads=True)      # where the workers are blocked
            for j, r in enumerate(runners):
                res = r.resident
                print(f"runner {j}: resident={res.stats() if res is not None else None} "
                      f"lock_held={r.r.lock.locked()} dev_lock_held={r.r.dev_lock.locked()}", flush=True)
            print("queue size", mb.q.qsize(), "busy", mb._busy, "health", mb.health(), flush=True)
            slow = sorted(calls, key=lambda c: -c[1])[:5]
            for c in slow:
                print(f"slow call: start +{c[0] - t0:.3f} s, {c[1]:.3f} s, rows {c[2]}, runner {c[3]}, "
                      f"resident before {c[4]} after {c[5]}", flush=True)
            print("calls", len(calls), "rows", sum(c[2] for c in calls), flush=True)
            rc = 2
        finally:
            mb.close()
        if rc:
            break
    return rc


if __name__ == "__main__":
    sys.exit(main(int(sys.argv[1]) if len(sys.argv) > 1 else 5))
