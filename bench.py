#!/usr/bin/env python3
"""Headline benchmark: ETA predictions/sec for the whole node (3-layer MLP, bf16 MFMA) plus the
p50 latency of a single ``/predict`` request through the serving stack.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``.  One rank per GPU over RCCL:
either the caller launches the ranks (``torch.distributed.run``, WORLD_SIZE set — it must equal N,
else exit 2), or, with WORLD_SIZE unset and N > 1, this script starts ``torch.distributed.run``
itself as a CHILD process before anything touches the GPU and exits with its code (fails loudly if
fewer than N GPUs are visible).  Each rank scores a fixed per-GPU batch of packed synthetic trip
records every step (weak scaling):

    step = the records of B requests go host -> HBM on the copy engine (one DMA on its own
           stream: large PCIe read TLPs, ~54 GB/s), then ONE fused featurize+MLP HIP launch
           (K1+K2) scores them from HBM and writes the predicted minutes straight into pinned host
           memory (zero-copy posted writes over the link's other direction).  Three slots are
           pipelined, so the copy of step k+1 overlaps the kernel of step k.

``--io zerocopy`` has the kernel read the records from pinned host memory itself (the PCIe read
direction then runs ~64-byte requests and tops out ~20 % lower, profiles/zerocopy_probe_r1.jsonl);
``--io host`` instead pipelines copy-engine H2D / kernel / D2H over three HIP streams;
``--io device`` scores HBM-resident records (kernel-only; reported as an extra field too).  K steps are timed between a barrier +
``torch.cuda.synchronize()`` on both sides; the max over ranks is reported by rank 0 as ONE JSON
line.  Weights are random-init (seeded), data is synthetic (no network, no checkpoints).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1 << 24,
                    help="rows per GPU per step (16M: the per-step DMA launch gap amortised; 8M is 2%% lower)")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--io", choices=["zerocopy", "hybrid", "host", "device"], default="hybrid",
                    help="zerocopy: the kernel reads pinned host records and writes pinned host "
                         "predictions over PCIe; host: copy-engine H2D/D2H pipeline; device: "
                         "records already resident in HBM")
    ap.add_argument("--rec", type=int, choices=[6, 8, 16], default=8,
                    help="wire record bytes per request (8: the serving format — the native front "
                         "end and the batcher send it for every batch it represents exactly; 16: "
                         "full record with epoch seconds; 6: lossy bulk research format) — "
                         "routest_amd/models/features.py")
    ap.add_argument("--variant", type=int, default=-1)
    ap.add_argument("--h2d-streams", type=int, default=1,
                    help="hybrid: split each step's record copy over this many copy streams")
    ap.add_argument("--p50", type=int, default=1, help="measure single-request p50 latency")
    ap.add_argument("--p50-requests", type=int, default=2000)
    ap.add_argument("--rec16-steps", type=int, default=10,
                    help="also time this many steps on full 16-byte records (extra JSON key)")
    ap.add_argument("--gcn-steps", type=int, default=30,
                    help="also time this many steps of the GCN route scorer (100k-node graph, 10k "
                         "routes per step over all ranks), replicated and row-partitioned with an "
                         "RCCL all-gather (extra JSON key 'gcn'; skipped on a shared GPU)")
    ap.add_argument("--train-steps", type=int, default=200,
                    help="also time this many data-parallel training steps of the same MLP on the "
                         "same ranks (64k rows per GPU, one flat-bucket RCCL all-reduce per step; "
                         "extra JSON key 'dp_training')")
    ap.add_argument("--train-batch-large", type=int, default=1 << 20,
                    help="also time the DP training probe at this many rows per GPU (extra JSON key "
                         "'dp_training_large_batch'; 0 skips)")
    ap.add_argument("--route-requests", type=int, default=10_000,
                    help="config 5: concurrent multi-stop requests per step over all ranks")
    ap.add_argument("--route-http-seconds", type=float, default=4.0,
                    help="route_optimizer.http: seconds of 1k-concurrency optimize_route load on the main port")
    ap.add_argument("--route-steps", type=int, default=3,
                    help="also time this many steps of the batched route optimizer (K5 + K6 + one "
                         "A* launch over MLP edge costs; extra JSON key 'route_optimizer'; skipped "
                         "on a shared GPU)")
    return ap.parse_args()


def main() -> None:
    a = parse_args()
    # rehearsal mode for 1-GPU boxes: every rank on GPU 0, gloo rendezvous (RCCL refuses two ranks
    # on one device).  The driver's N-GPU runs never set it: one rank per GPU over RCCL.  Tagged
    # "shared_gpu" in the JSON so a rehearsal number cannot be read as a whole-node number.
    from routest_amd.parallel.launch import ensure_ranks, share_gpu
    share = share_gpu()
    world = ensure_ranks(a.gpus, __file__)    # may run the ranks as a child and exit
    import numpy as np
    import torch
    import torch.distributed as dist

    from routest_amd.parallel.dp import allreduce_scalars
    from routest_amd.utils import bench_schema

    import datetime
    from routest_amd.utils.bench_guard import SectionAborted, SectionGuard, env_timeout_s, raise_if_injected

    rank = int(os.environ.get("RANK", "0"))
    local_rank = 0 if share else int(os.environ.get("LOCAL_RANK", "0"))
    # a collective that never completes (a peer died, an RCCL hang) ends in an error after this
    # long instead of running into the driver's limit with no JSON line printed
    pg_timeout = datetime.timedelta(seconds=env_timeout_s("ROUTEST_BENCH_PG_TIMEOUT_S", 180.0))
    # ... and what happens then: CleanUpOnly (2) aborts the hung RCCL communicator, so the waiting
    # stream completes with an error and the section reports it under the guard; torch's default
    # (3, SkipCleanUp) tears the whole process down from the watchdog thread — no JSON line
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
    if world > 1:
        torch.cuda.set_device(local_rank)
        if share:
            dist.init_process_group("gloo", timeout=pg_timeout)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), timeout=pg_timeout)
    # every extra section runs under the guard (routest_amd/utils/bench_guard.py): a failure on one
    # rank becomes an {"error": ...} key on every rank, agreed on over a gloo side group before any
    # rank enters a collective the failed one would never reach
    guard = SectionGuard(world, rank, timeout_s=env_timeout_s("ROUTEST_BENCH_HOLD_TIMEOUT_S", 900.0))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    from routest_amd.parallel.affinity import bind_to_gpu_numa
    numa = bind_to_gpu_numa(local_rank)   # pinned request buffers on the GPU's local NUMA node

    from routest_amd.data.synth import synth_records
    from routest_amd.models.features import records_to_features
    from routest_amd.models.mlp3 import EtaMLP
    from routest_amd.models.features import records_to_compact6, records_to_wire8
    from routest_amd.ops.eta_mlp import (EtaMlpKernel, records6_to_tensor, records8_to_tensor,
                                         records_to_tensor)

    torch.manual_seed(1234)
    model = EtaMLP(a.hidden)
    norm_rec, norm_y = synth_records(65536, seed=11)
    model.fit_normalization(records_to_features(norm_rec), norm_y)
    kern = EtaMlpKernel(model, dev, variant=a.variant)

    B = a.batch
    rec, _ = synth_records(B, seed=100 + rank)

    def wire(nbytes: int) -> torch.Tensor:
        if nbytes == 8:
            # the same exactness-guarded packer the service runs (features.records_to_wire8 ==
            # csrc/runtime/rt_core.h pack_wire8): pickup hours since the batch's base Monday, the
            # kernel derives weekday/hour; the synthetic pickups carry minutes/seconds like real
            # ISO timestamps and integer ages, so the whole batch is representable
            r8 = records_to_wire8(rec)
            assert r8 is not None, "synthetic batch not representable as 8-byte wire records"
            return records8_to_tensor(r8).pin_memory()
        return (records6_to_tensor(records_to_compact6(rec)) if nbytes == 6 else
                records_to_tensor(rec)).pin_memory()

    nbuf = 3
    h2d_s = torch.cuda.Stream(dev)      # PCIe host->device
    comp_s = torch.cuda.Stream(dev)     # fused featurize+MLP kernel
    d2h_s = torch.cuda.Stream(dev)      # PCIe device->host (other direction, overlaps H2D)
    h2d_extra = [torch.cuda.Stream(dev) for _ in range(max(0, a.h2d_streams - 1))]
    host_out = [torch.empty(B, dtype=torch.float32).pin_memory() for _ in range(nbuf)]

    class Pipeline:
        """Three slots of (records in HBM, minutes out); ``step(i)`` enqueues step i."""

        def __init__(self, host_rec: torch.Tensor):
            self.host_rec = host_rec
            self.dev_rec = [torch.empty_like(host_rec, device=dev) for _ in range(nbuf)]
            self.dev_out = [None] * nbuf
            self.h2d_done = [torch.cuda.Event() for _ in range(nbuf)]
            self.comp_done = [torch.cuda.Event() for _ in range(nbuf)]
            self.d2h_done = [torch.cuda.Event() for _ in range(nbuf)]
            self.h2d_parts = [[torch.cuda.Event() for _ in range(nbuf)] for _ in range(a.h2d_streams)]
            for i in range(nbuf):
                self.dev_rec[i].copy_(host_rec)
            torch.cuda.synchronize()

        def step(self, i: int) -> None:
            k = i % nbuf
            host_rec, dev_rec, dev_out = self.host_rec, self.dev_rec, self.dev_out
            comp_done = self.comp_done
            if a.io == "zerocopy":
                with torch.cuda.stream(comp_s):
                    kern.forward_hostio(host_rec, host_out[k])
            elif a.io == "hybrid":
                # records in by DMA (large PCIe read TLPs), minutes out as the kernel's own posted
                # writes over the other link direction
                n = len(h2d_extra) + 1
                for j, cs in enumerate([h2d_s] + h2d_extra):
                    lo, hi = B * j // n, B * (j + 1) // n
                    with torch.cuda.stream(cs):
                        cs.wait_event(comp_done[k])         # slot k's records consumed
                        dev_rec[k][lo:hi].copy_(host_rec[lo:hi], non_blocking=True)
                        self.h2d_parts[j][k].record(cs)
                with torch.cuda.stream(comp_s):
                    for j in range(n):
                        comp_s.wait_event(self.h2d_parts[j][k])
                    kern.forward_hostio(dev_rec[k], host_out[k])
                    comp_done[k].record(comp_s)
            elif a.io == "host":
                with torch.cuda.stream(h2d_s):
                    h2d_s.wait_event(comp_done[k])          # slot k's records consumed
                    dev_rec[k].copy_(host_rec, non_blocking=True)
                    self.h2d_done[k].record(h2d_s)
                with torch.cuda.stream(comp_s):
                    comp_s.wait_event(self.h2d_done[k])
                    comp_s.wait_event(self.d2h_done[k])     # slot k's previous output drained
                    dev_out[k] = kern(dev_rec[k])
                    comp_done[k].record(comp_s)
                with torch.cuda.stream(d2h_s):
                    d2h_s.wait_event(comp_done[k])
                    host_out[k].copy_(dev_out[k], non_blocking=True)
                    self.d2h_done[k].record(d2h_s)
            else:
                with torch.cuda.stream(comp_s):
                    dev_out[k] = kern(dev_rec[k])

        def timed(self, warmup: int, steps: int) -> float:
            """``warmup`` untimed steps, then ``steps`` timed ones between barrier + synchronize
            on both sides; returns the max over ranks of the elapsed seconds."""
            for i in range(warmup):
                self.step(i)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            # per-step completion times (an event on the compute stream after each step; event
            # records are asynchronous and cost nothing on the timed path)
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
            evs[0].record(comp_s)
            t0 = time.perf_counter()
            for i in range(steps):
                self.step(warmup + i)
                evs[i + 1].record(comp_s)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            d = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(1, steps))
            self.step_ms = ({"p50": d[len(d) // 2], "p90": d[int(len(d) * 0.9)], "min": d[0], "max": d[-1]}
                            if d else None)
            if world > 1:
                (el,) = allreduce_scalars([el], dev, "max")
            return el

        def last_output(self, i: int) -> torch.Tensor:
            k = i % nbuf
            if a.io == "device":
                return self.dev_out[k].float().cpu()
            return host_out[k].clone()

    pipe = Pipeline(wire(a.rec))
    # GPU clocks ramp over the first ~20 launches (kernel 2.3 -> 1.6 ms in
    # profiles/headline_trace_r2.md): spin the kernel on HBM-resident records before the warmup
    for _ in range(40):
        kern(pipe.dev_rec[0])
    torch.cuda.synchronize()
    elapsed = pipe.timed(a.warmup, a.steps)
    step_dist = pipe.step_ms          # intervals between consecutive steps' kernel completions

    # the link bound: the record DMA alone, same bytes, same stream (what the step cannot beat)
    h2d_only_ms = None
    if a.io == "hybrid":
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(h2d_s):
            e0.record(h2d_s)
            for _ in range(10):
                pipe.dev_rec[1].copy_(pipe.host_rec, non_blocking=True)
            e1.record(h2d_s)
        torch.cuda.synchronize()
        h2d_only_ms = e0.elapsed_time(e1) / 10

    # verify the headline kernel's own output from the last timed step (not a separate small
    # launch): every row finite, and a 64k-row slice against the fp32 model and the bf16 emulation
    # of the kernel on the same (wire-format-decoded) features
    from routest_amd.ops.eta_mlp import emulate_kernel, featurize_torch
    got = pipe.last_output(a.warmup + a.steps - 1)
    from routest_amd.utils.faults import active_faults
    if "bench_corrupt_output" in active_faults():     # test hook: the check must catch this
        got[0] = float("nan")
        got[1:64] += 1e3
    ok = bool(torch.isfinite(got).all().item())
    nchk = min(B, 65536)
    rec_chk = pipe.host_rec[:nchk]
    with torch.no_grad():
        ref32 = model.float().cpu()(featurize_torch(rec_chk)).reshape(-1)
    emu = emulate_kernel(kern.packed.to("cpu"), rec_chk, kern._pick(B)).reshape(-1)
    spread = float((ref32 - ref32.mean()).abs().mean()) + 1e-6
    err_fp32 = float((got[:nchk] - ref32).abs().max()) / spread
    err_emu = float((got[:nchk] - emu).abs().max()) / spread
    ok = ok and err_emu < 0.05 and err_fp32 < 0.25

    # device-only throughput of the fused kernel on the same batch (reported alongside)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        kern(pipe.dev_rec[0])
    ev0.record()
    for _ in range(30):
        kern(pipe.dev_rec[0])
    ev1.record()
    torch.cuda.synchronize()
    kernel_preds_per_s = B * 30 / (ev0.elapsed_time(ev1) / 1e3)

    # the same pipeline on full 16-byte records (epoch seconds: weekday/hour resolved by the
    # kernel itself, float age and distance — no lossy packing), reported as an extra key
    rec16_value = None
    if a.rec != 16 and a.rec16_steps > 0:
        del pipe

        def rec16_section():
            pipe16 = Pipeline(wire(16))
            guard.checkpoint()                      # (timed() barriers on the main group)
            el16 = pipe16.timed(min(a.warmup, 3), a.rec16_steps)
            del pipe16
            return B * a.rec16_steps * world / el16
        rec16_value = guard.run("rec16", rec16_section)
        if isinstance(rec16_value, dict):           # {"error": ...}: reported, not a rate
            rec16_value = None

    # config 3 on the same ranks: the fused DP training step (forward + MSE gradient + dgrad in
    # one kernel, split-K weight gradients, one flat-bucket all-reduce, fused AdamW + re-pack)
    def train_probe(comm=None, tB: int = 65536):
        from routest_amd.train.fused import FusedMlp3Trainer
        torch.manual_seed(4321)                 # identical initial parameters on every rank
        tmodel = EtaMLP(a.hidden)
        tmodel.fit_normalization(records_to_features(norm_rec), norm_y)
        trec, ty = synth_records(tB, seed=300 + rank)
        trt = records_to_tensor(trec).to(dev)
        tr = FusedMlp3Trainer(tmodel, dev, tB, tB * world, lr=1e-3, allreduce=world > 1, comm=comm)
        yn = tr.normalize_targets(torch.from_numpy(ty).to(dev))
        for _ in range(20):                     # (clocks settle: 5 warm steps read ~5 % slow at 64k)
            guard.checkpoint()                  # (each step all-reduces the gradient bucket)
            tr.step(trt, yn)
        torch.cuda.synchronize()
        if comm is not None and not guard.agree(not comm.C.comm_error(comm.h)):
            return {"error": "one-shot all-reduce: a peer wait timed out during warmup"}
        # one rank: the whole step (4 kernels, no host work, no sync) replays as ONE captured HIP graph
        # — the launch-bound inner loop the design captures instead of tracing.  Multi-rank steps
        # stay eager (their all-reduce goes through RCCL / gloo / the one-shot path)
        step = lambda: tr.step(trt, yn)  # noqa: E731
        launch, probe_launch = "eager", None
        if world == 1 and comm is None and os.environ.get("ROUTEST_BENCH_TRAIN_GRAPH", "1") != "0":
            try:
                cs = torch.cuda.Stream(dev)
                cs.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(cs):
                    for _ in range(3):
                        tr.step(trt, yn)
                torch.cuda.current_stream(dev).wait_stream(cs)
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    tr.step(trt, yn)
                for _ in range(3):
                    graph.replay()
                torch.cuda.synchronize()
                # keep whichever launch runs the step faster on this box (run r6h: graph replay
                # 71.4 vs eager 67.6 us; round 5: 67.1 vs 70.6) — both execute the identical step
                def _rate(fn, n=50):
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    for _ in range(n):
                        fn()
                    torch.cuda.synchronize()
                    return (time.perf_counter() - t) / n * 1e3
                probe_launch = {"eager_ms": _rate(step), "graph_ms": _rate(graph.replay)}
                if probe_launch["graph_ms"] < probe_launch["eager_ms"]:
                    step, launch = graph.replay, "hip graph (one capture of the whole step, replayed)"
            except Exception:  # noqa: BLE001 - eager launches are always valid
                torch.cuda.synchronize()
        guard.checkpoint()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.train_steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        tel = time.perf_counter() - t0
        guard.checkpoint()
        if world > 1:
            (tel,) = allreduce_scalars([tel], dev, "max")
        loss = float(tr.sq_err.sum().item()) / tB
        res = bench_schema.dp_training(
            tB * world * a.train_steps / tel, tel / a.train_steps * 1e3, tB, world, a.train_steps,
            ("none" if world == 1 else "gloo (shared GPU)" if share and comm is None
             else "RCCL, one flat fp32 bucket" if comm is None else
             "one-shot over IPC-mapped peer HBM (csrc/comm.hip), one flat fp32 bucket"), loss, launch=launch,
            launch_probe_ms=probe_launch)
        if comm is not None:
            res["comm_error"] = not guard.agree(not comm.C.comm_error(comm.h))
            # every rank must hold the same parameters after the identical reduced updates
            ph = float(tr.P.double().sum())
            guard.checkpoint()
            (lo,) = allreduce_scalars([ph], dev, "min")
            (hi,) = allreduce_scalars([ph], dev, "max")
            res["params_identical_across_ranks"] = bool(lo == hi)
        del tr, trt
        return res

    train_res = guard.run("train", train_probe) if a.train_steps > 0 else None
    # the same step at 1M rows per GPU (16 MB of records — HBM is never the limit): the fixed
    # per-step costs (slab reduction, AdamW, launch gaps, the all-reduce) amortised over 16x the rows
    train_big_res = (guard.run("train_large", train_probe, tB=a.train_batch_large)
                     if a.train_steps > 0 and a.train_batch_large > 0 else None)

    # the same training step with the native one-shot all-reduce (one hop over all 7 xGMI links at
    # once, instead of RCCL's latency-bound ring at this 296 KB bucket).  Set-up failures and peer
    # timeouts are agreed on by every rank before anything else runs, so no rank is left waiting.
    train_os_res = None
    devcomm = None
    if a.train_steps > 0 and world > 1 and os.environ.get("ROUTEST_BENCH_ONESHOT", "1") != "0":
        from routest_amd.parallel.comm import DeviceComm
        holder = {}

        def oneshot_section():
            err = None
            try:
                guard.checkpoint()               # (the IPC set-up exchanges handles over the group)
                holder["comm"] = DeviceComm(dev, use_rccl=False)
                os_ok = holder["comm"].oneshot
            except SectionAborted:
                raise
            except Exception as e:  # noqa: BLE001 - reported, never fatal for the headline
                os_ok, err = False, repr(e)[:200]
            # (os_ok, not ok: `ok` holds the headline output check reported as "finite" / exit 3)
            if not guard.agree(os_ok):
                holder.pop("comm", None)
                return {"error": err or "one-shot set-up failed on a peer rank"}
            return train_probe(holder["comm"])
        train_os_res = guard.run("oneshot", oneshot_section)
        devcomm = holder.get("comm")
        if devcomm is not None and ("error" in train_os_res or train_os_res.get("comm_error")):
            # (agreed on by every rank inside the section): no further one-shot use
            torch.cuda.synchronize()
            devcomm.close()
            devcomm = None

    # whole-node runs: what the xGMI links delivered, measured on the same ranks right after the
    # timed region (RCCL all-reduce / all-gather sweep; extra JSON key, outside the timing)
    coll = None
    if world > 1 and not share and os.environ.get("ROUTEST_BENCH_COLLECTIVES", "1") != "0":
        # RCCL on the process group bench.py already holds, plus the one-shot all-reduce when its
        # set-up and training probe succeeded on every rank: every decision here depends only on
        # state all ranks agreed on, so no rank can be left waiting on a step another one skipped
        from routest_amd.parallel.collective_probe import sweep
        coll = guard.run("collectives", sweep, dev, native=devcomm, checkpoint=guard.checkpoint)
        if isinstance(coll, dict):
            coll = [coll]                       # schema: a list whose first row carries "error"

    # config 4 on the same ranks: the 2-layer GCN scorer, graph replicated on every GPU (no
    # collective) and row-partitioned (each rank runs 1/N of the nodes, RCCL all-gather of Z).  The
    # shared-GPU rehearsal runs every mode too (its "partition" gathers through gloo via host memory)
    gcn_res = None
    g = None
    if a.gcn_steps > 0:
        from routest_amd.data.graph import synth_road_graph
        from routest_amd.models.gcn import GcnScorer, GcnScorerHip, routes_to_csr
        g = synth_road_graph(100_000, seed=0)

        def gcn_section():
            gm = GcnScorer(seed=0)
            rng = np.random.default_rng(rank)
            nroutes = 10_000 // world
            walks = []
            for _ in range(nroutes):
                v = int(rng.integers(0, g.num_nodes))
                path = [v]
                for _ in range(int(rng.integers(50, 300))):
                    nb = g.indices[g.indptr[v]:g.indptr[v + 1]]
                    v = int(nb[rng.integers(0, len(nb))])
                    path.append(v)
                walks.append(path)
            ptr, nodes = routes_to_csr(walks)
            ptr_t, nodes_t = torch.from_numpy(ptr).to(dev), torch.from_numpy(nodes).to(dev)
            res = bench_schema.gcn_section(g.num_nodes, g.num_edges, nroutes * world)
            modes = list(bench_schema.GCN_MODES_N if world > 1 else bench_schema.GCN_MODES_1)
            if world > 1 and devcomm is not None:
                modes.append(bench_schema.GCN_MODE_ONESHOT)   # Z gathered over IPC-mapped peer HBM in one hop
            for mode in modes:
                guard.checkpoint()
                hip = GcnScorerHip(gm, g, dev, mode=mode.split("_")[0], rank=rank, world=world,
                                   comm=devcomm if mode.endswith("oneshot") else None)

                def gstep():
                    hip.node_delays()
                    return hip.score_routes(ptr_t, nodes_t)
                for _ in range(5):
                    guard.checkpoint()          # (partition modes all-gather inside the step)
                    gstep()
                torch.cuda.synchronize()
                guard.checkpoint()
                if world > 1:
                    dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.gcn_steps):
                    gstep()
                torch.cuda.synchronize()
                if world > 1:
                    dist.barrier()
                torch.cuda.synchronize()
                gel = time.perf_counter() - t0
                guard.checkpoint()
                if world > 1:
                    (gel,) = allreduce_scalars([gel], dev, "max")
                bench_schema.gcn_mode(res, mode, gel, a.gcn_steps, nroutes * world)
                del hip
            return res
        gcn_res = guard.run("gcn", gcn_section)

    # config 5 on the same ranks: 10k concurrent multi-stop requests sharded over the ranks, each
    # step CCH road-metre matrices + K6 greedy for all of a rank's requests, then every trip leg as
    # one CCH query with its path unpacked, over MLP-learned edge times (no collective; timing max
    # over ranks).  The routing context's customization happens once, outside the timed steps, and
    # is reported as `context_customize_ms` (a fresh context, measured separately).  The shared-GPU
    # rehearsal runs it too: each rank on GPU 0 with its share of the requests, reductions via gloo.
    route_res = None
    route_cost = None
    route_router = None
    route_model = None
    if a.route_steps > 0:
        from routest_amd.data.graph import synth_road_graph
        from routest_amd.routing.bulk import BulkRouteStep
        from routest_amd.routing.cch import RoadRouter, RouteContext
        from routest_amd.routing.graph import edge_costs
        from routest_amd.serve.eta_service import default_model
        held = {}

        def route_section():
            # set-up is per rank (no collective); a failure on any rank is agreed on (the
            # checkpoint) before the timed steps' barrier
            gr = g if g is not None else synth_road_graph(100_000, seed=0)
            torch.manual_seed(0)
            rmodel = default_model(hidden=a.hidden, steps=200)
            cost = edge_costs(gr, rmodel, device=dev)
            t0 = time.perf_counter()
            router = RoadRouter(gr, rmodel, device=dev)
            topo_s = time.perf_counter() - t0
            # a routing context built from scratch on the GPU: ETA-model edge costs + customization
            t0 = time.perf_counter()
            router.metric(RouteContext(weather=1, congestion=3, weekhour=4 * 24 + 18))
            ctx_ms = (time.perf_counter() - t0) * 1e3
            ctx_info = dict(router.last_metric)
            bulk = BulkRouteStep(gr, cost, dev, a.route_requests // world, seed=100 + rank, router=router)
            bulk.step()
            torch.cuda.synchronize()
            guard.checkpoint()
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            legs, unfound = 0, 0
            for _ in range(a.route_steps):
                nl, _, st, _ = bulk.step()
                legs += nl
                unfound += (st != 0).sum()          # device-side count, read once after the loop
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            rel = time.perf_counter() - t0
            unfound = int(unfound)
            guard.checkpoint()
            if world > 1:
                rel, legs, unfound = bench_schema.reduce_route_stats(rel, legs, unfound, dev)
            R = a.route_requests // world * world
            held.update(graph=gr, cost=cost, router=router, model=rmodel)
            del bulk
            return bench_schema.route_section(R, a.route_steps, rel, legs, unfound, gr.num_nodes, ctx_ms,
                                              ctx_info, topo_s, router.stats(), world)
        route_res = guard.run("route", route_section)
        if "error" not in route_res:
            g, route_cost, route_router, route_model = held["graph"], held["cost"], held["router"], held["model"]

    p50_ms = p99_ms = None
    p50_fastapi_ms = None
    p50_py_ms = None
    conc = None
    serving_error = None
    if a.p50 and rank == 0:
        # (rank 0 alone; ranks 1..N-1 wait at guard.hold() below.  A failure here is reported as
        # "serving_error" and the line still prints)
        try:
            raise_if_injected("serving", rank)
            # (1) headline p50 on the MAIN port of the stack `routest serve` runs (serve/frontend.py
            #     ServingStack): real HTTP/1.1 over loopback (keep-alive) to the native front end
            #     (csrc/native_server.hip): socket -> C++ JSON pack -> fused HIP kernel on this GPU
            #     (zero-copy) -> C++ response formatting; the FastAPI app sits behind it for the long
            #     tail.  Same endpoint semantics as the FastAPI handler (byte-identical bodies,
            #     tests/test_frontend_gpu.py).  With the road graph of config 5 loaded, the same port
            #     also serves the route_optimizer HTTP variant below.
            import http.client
            from routest_amd.api.app import build_services, create_app
            from routest_amd.config import load_settings
            from routest_amd.serve.eta_service import EtaService
            from routest_amd.serve.frontend import ServingStack, route_pipelines_for
            from routest_amd.serve.loadgen import native_route_load, route_payloads
            body = {"summary": {"distance": 12345}, "pickup_time": "2026-10-15T08:30:00",
                    "driver_age": 34, "weather": "Sunny", "traffic": "Medium"}
            raw = json.dumps(body).encode()
            hdr = {"Content-Type": "application/json"}
            prov = None
            if g is not None and route_cost is not None:
                from routest_amd.routing.graph import GraphProvider
                # context-aware road provider sharing the bench's router (the customized contexts)
                prov = GraphProvider(g, None, device=dev, eta_model=route_model)
                prov._routers[str(torch.device(dev))] = route_router
            # native route services per GPU (ROUTEST_ROUTE_PIPELINES, config.py route_pipelines)
            pipes = max(0, int(os.environ.get("ROUTEST_ROUTE_PIPELINES", "0")))
            ss = load_settings(env={}, dotenv_path=None, devices=[local_rank], warm_scorer=False,
                               route_pipelines=pipes)
            sv = build_services(ss, eta=EtaService(model, devices=[local_rank]), provider=prov, store=None)
            with ServingStack(sv, create_app(sv), model, [local_rank], threads=8) as srv:
                # native closed-loop client (csrc/runtime/http_client.h): one keep-alive connection,
                # one request in flight — the client adds ~1 us instead of http.client's ~30 us
                from routest_amd.ops import _ext
                rtm = _ext.runtime(required=True)
                r1 = rtm.http_load(srv.port, 1, 30.0, "/api/predict_eta", raw.decode(), 1,
                                   a.p50_requests, 200)
                assert r1["errors"] == 0 and r1["requests"] >= a.p50_requests, r1
                lat = r1["latencies_us"]
                p50_ms = float(lat[len(lat) // 2]) * 1e-3
                p99_ms = float(lat[int(len(lat) * 0.99) - 1]) * 1e-3
                # the same with Python's http.client (what a Python caller would see)
                conn = http.client.HTTPConnection("127.0.0.1", srv.port)
                latp = []
                for j in range(a.p50_requests // 2 + 200):
                    t1 = time.perf_counter()
                    conn.request("POST", "/api/predict_eta", body=raw, headers=hdr)
                    r = conn.getresponse()
                    r.read()
                    if j >= 200:
                        latp.append(time.perf_counter() - t1)
                    assert r.status == 200
                latp.sort()
                p50_py_ms = latp[len(latp) // 2] * 1e3
                # 16 concurrent single-item clients (separate connections; the reactors batch them)
                r16 = rtm.http_load(srv.port, 16, 2.0, "/api/predict_eta", raw.decode(), 4, 0, 50)
                assert r16["errors"] == 0, r16
                conc = r16["requests"] / r16["seconds"]
                # config 5 as a service: 1k concurrent multi-stop optimize_route requests on the same
                # port — CCH road matrices + K6 + CCH legs + path copy-out + C++ GeoJSON (maneuvers)
                if prov is not None and route_res is not None and srv.front.routes:
                    route_res["http"] = native_route_load(srv, route_payloads(g.lat, g.lon, 1000, seed=1), 1000,
                                                          a.route_http_seconds)
                    route_res["http"]["route_pipelines_per_gpu"] = route_pipelines_for(sv)
            sv.eta.close()
            # the dashboard's own request (F02 verbatim: use_ml_eta, context, meta, driver_age) at 1k
            # concurrency on the same port, every answer persisted into a SQLite store on disk — the
            # canonical product path of /api/optimize_route (RO/Flaskr/routes.py:89-127)
            if (prov is not None and isinstance(route_res, dict) and "error" not in route_res
                    and a.route_http_seconds > 0):
                import tempfile
                from routest_amd.serve.loadgen import f02_payloads
                from routest_amd.store.store import SQLiteStore
                with tempfile.TemporaryDirectory(prefix="routest-bench-") as td:
                    store = SQLiteStore(os.path.join(td, "routest.db"))
                    ids = [loc["id"] for loc in store.locations()]
                    sv2 = build_services(ss, eta=EtaService(model, devices=[local_rank]), provider=prov, store=store)
                    with ServingStack(sv2, create_app(sv2), model, [local_rank], threads=8) as srv2:
                        if srv2.front.routes:
                            r2 = native_route_load(srv2, f02_payloads(g.lat, g.lon, 1000, seed=2, location_ids=ids),
                                                   1000, a.route_http_seconds)
                            r2["store"] = "sqlite file (WAL, synchronous=NORMAL), group commit per flush"
                            r2["route_pipelines_per_gpu"] = route_pipelines_for(sv2)
                            route_res["http_f02"] = r2
                    sv2.eta.close()
                    store.close()

            # (2) the FastAPI app in-process over ASGI (like the reference's Flask test-client figure)
            import asyncio
            import httpx
            from routest_amd.api.app import build_services, create_app
            from routest_amd.config import load_settings
            from routest_amd.serve.eta_service import EtaService
            s = load_settings(env={}, dotenv_path=None, devices=[local_rank])
            app = create_app(build_services(s, eta=EtaService(model, devices=[local_rank]), store=None))

            async def _lat():
                out = []
                async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app),
                                             base_url="http://bench") as c:
                    for j in range(a.p50_requests + 200):
                        t1 = time.perf_counter()
                        r = await c.post("/api/predict_eta", json=body)
                        dt_ = time.perf_counter() - t1
                        assert r.status_code == 200, r.text
                        if j >= 200:
                            out.append(dt_)
                return out
            lat2 = sorted(asyncio.run(_lat()))
            p50_fastapi_ms = lat2[len(lat2) // 2] * 1e3
            app.state.services.eta.close()
        except Exception as e:  # noqa: BLE001 - the headline line must still print
            import traceback
            traceback.print_exc()
            serving_error = repr(e)[:300]

    if rank == 0:
        preds = B * a.steps * world
        value = preds / elapsed
        out = {
            "metric": "ETA preds/sec (whole node) + p50 /predict latency, 3-layer MLP bf16",
            "value": value,
            "unit": "predictions/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            # BASELINE.md publishes no reference number; its survey-measured CPU calibration points
            # are ~359k preds/s (bulk tree-ensemble proxy, 8 threads) and p50 0.603 ms (Flask)
            "vs_survey_bulk_cpu_proxy": value / 359e3,
            "p50_vs_survey_flask": (0.603 / p50_ms) if p50_ms else None,
            "dtype": "bf16",
            "data": "synthetic (seeded trip records, random-init weights)",
            "config": {"model": f"mlp3 12->{a.hidden}->{a.hidden}->1 (fused featurize+MLP HIP kernel)",
                       "global_batch": B * world, "seq_len": None,
                       "parallelism": f"dp{world} (inference sharding, 1 replica/GPU)",
                       "io": a.io, "record_bytes": a.rec, "numa_node": numa},
            "kernel_only_preds_per_s_per_gpu": kernel_preds_per_s,
            "h2d_copy_only_ms": h2d_only_ms,
            "step_ms_distribution": step_dist,
            "step_vs_h2d_copy_only": (h2d_only_ms / (elapsed / a.steps * 1e3)) if h2d_only_ms else None,
            "p50_predict_ms": p50_ms,
            "p99_predict_ms": p99_ms,
            "p50_path": "main port of the serving stack (`routest serve`: native front end + FastAPI app behind it): "
                        "HTTP/1.1 loopback keep-alive POST /api/predict_eta -> C++ reactor -> fused HIP kernel; "
                        "native closed-loop client",
            "p50_python_client_ms": p50_py_ms,
            "p50_fastapi_asgi_ms": p50_fastapi_ms,
            "http_concurrent16_req_per_s": conc,
            "preds_per_s_rec16": rec16_value,
            "record_format": {6: "6 B packed (lossy research format): distance 1/8 m, integer age 0-127, host weekday/hour",
                              8: "8 B wire record = the serving format (native front end, batcher): fp32 distance, "
                                 "fp16 age (exactness-guarded, else 16 B), pickup hours since the batch's base "
                                 "Monday; weekday/hour featurised by the kernel; bit-identical predictions to 16 B",
                              16: "16 B full: fp32 distance, fp32 age, epoch seconds (kernel featurises)"}[a.rec],
            "shared_gpu": bool(share and world > 1),
            "collectives": coll,
            "dp_training": train_res,
            "dp_training_oneshot": train_os_res,
            "dp_training_large_batch": train_big_res,
            "gcn": gcn_res,
            "route_optimizer": route_res,
            "serving_error": serving_error,
            "check_max_err_vs_emulation": err_emu,
            "check_max_err_vs_fp32": err_fp32,
            "finite": ok,
        }
        out["schema_problems"] = bench_schema.problems(out)
        print(json.dumps(out), flush=True)
    # every rank meets on the gloo side group (ranks 1..N-1 have waited here while rank 0 served),
    # then the communicators are torn down together
    guard.hold()
    if devcomm is not None:
        torch.cuda.synchronize()
        devcomm.close()
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        print("bench.py: output check failed", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
