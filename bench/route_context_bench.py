"""Routing contexts under load on the main port (verdict r4 item 2 "done when"): the dashboard's
request (F02 payloads, ``serve/loadgen.py f02_payloads``: ML ETA, ``meta``, every answer persisted to
a SQLite file) at 1k closed-loop connections, with the routing context varied.

Phases (``--phases``, one JSON line each, then a summary line):

* ``single``   — every request under one explicit context (``pickup_time`` fixed): the reference p99.
* ``cycle64``  — 64 distinct (weather, traffic, pickup_time) contexts, request ``i`` under context
  ``i % 64``: a cold window (the 64 contexts are built by the router's background builder while
  the load runs), then the steady state (all 64 cached).  ``p99_vs_single`` is the steady ratio.
* ``hour`` / ``hour_noprefetch`` — requests routed at "now" (no ``pickup_time``) across an hour
  boundary: the route service's clock is shifted (``ROUTEST_ROUTE_CLOCK_SKEW_S``) so the boundary
  falls ~12 s into a run of 1-second windows; per-window p50 / p99 / max.  With prefetch (default
  ``ROUTEST_CCH_PREFETCH_MIN`` = 10) the next hour's contexts are built before the boundary; the
  ``_noprefetch`` run shows what the boundary costs without it (every request of the new hour
  waits for one build).
* ``fresh``    — (meant for ``--nodes 1000000``) a cached context under load in 0.5-second windows
  while a side thread sends requests under four contexts never seen: the cached requests' windows
  during the builds against the ones before.

    python bench/route_context_bench.py --phases single,cycle64,hour,hour_noprefetch
    python bench/route_context_bench.py --nodes 1000000 --concurrency 256 --phases fresh
"""
import argparse
import http.client
import json
import os
import sys
import tempfile
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

WEATHERS = ("Sunny", "Cloudy", "Windy", "Stormy")
TRAFFICS = ("Low", "Medium", "High", "Jam")
PICKUPS = ("2025-09-01T07:20:00", "2025-09-02T12:40:00", "2025-09-03T17:05:00", "2025-09-04T22:30:00")


def emit(d):
    print(json.dumps(d), flush=True)


def pct(lat_us, q):
    if not len(lat_us):
        return None
    return round(float(lat_us[min(len(lat_us) - 1, max(0, int(len(lat_us) * q) - (1 if q >= 0.99 else 0)))]) / 1e3, 3)


class Bench:
    def __init__(self, a):
        from routest_amd.data.graph import synth_road_graph
        from routest_amd.ops import _ext
        from routest_amd.routing.graph import GraphProvider
        from routest_amd.serve.eta_service import default_model
        self.a = a
        self.dev = torch.device("cuda", 0)
        t0 = time.time()
        self.g = synth_road_graph(a.nodes, seed=0)
        self.model = default_model(steps=50)
        self.prov = GraphProvider(self.g, None, device=self.dev, eta_model=default_model(hidden=64, steps=50))
        self.rt = _ext.runtime(required=True)
        self.td = tempfile.TemporaryDirectory(prefix="routest-ctx-")
        emit({"stage": "setup", "nodes": self.g.num_nodes, "s": round(time.time() - t0, 2)})

    def stack(self, env):
        """A serving stack (native front end + route service + SQLite store) built under ``env``
        (the route service reads its knobs at construction)."""
        from routest_amd.api.app import build_services, create_app
        from routest_amd.config import load_settings
        from routest_amd.serve.eta_service import EtaService
        from routest_amd.serve.frontend import ServingStack
        from routest_amd.store.store import SQLiteStore
        # (kept set while the stack runs: the route service may be constructed after this returns)
        self._env_old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        store = SQLiteStore(os.path.join(self.td.name, f"routest{len(os.listdir(self.td.name))}.db"))
        ss = load_settings(env={}, dotenv_path=None, devices=[0], warm_scorer=False)
        sv = build_services(ss, eta=EtaService(self.model, devices=[0]), provider=self.prov, store=store)
        st = ServingStack(sv, create_app(sv), self.model, [0], threads=8)
        assert st.front.routes, "native route service not running"
        return st, sv, store

    def close(self, st, sv, store):
        st.close()
        sv.eta.close()
        store.close()
        for k, v in getattr(self, "_env_old", {}).items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        self._env_old = {}

    def payloads(self, n, ctx_of, store, seed=2):
        from routest_amd.serve.loadgen import f02_payloads
        ids = [loc["id"] for loc in store.locations()]
        reqs = f02_payloads(self.g.lat, self.g.lon, n, seed=seed, location_ids=ids)
        for i, r in enumerate(reqs):
            c = ctx_of(i)
            if c is not None:
                r["context"] = c
        return [json.dumps(r) for r in reqs]

    def window(self, st, bodies, conc, secs):
        paths = ["/api/optimize_route"] * len(bodies)
        # (the first response of each connection is not recorded: it includes the connect and the
        # arrival of every connection's first request at once — loadgen.native_route_load does the same)
        r = self.rt.http_load_multi(st.port, conc, secs, paths, bodies, 8, 0, 1)
        lat = r["latencies_us"]
        return {"s": round(r["seconds"], 3), "requests": int(r["requests"]), "errors": int(r["errors"]),
                "req_per_s": round(r["requests"] / max(r["seconds"], 1e-9), 1), "p50_ms": pct(lat, 0.5),
                "p99_ms": pct(lat, 0.99), "max_ms": round(float(lat[-1]) / 1e3, 3) if len(lat) else None}

    @staticmethod
    def delta(st, s0):
        s1 = st.front.stats()
        keys = ("route_flushes", "route_ctx_deferred", "route_us_ctx_wait", "route_ctx_prefetched",
                "route_contexts_built", "route_service_fallbacks", "route_persisted")
        out = {k: s1.get(k, 0) - s0.get(k, 0) for k in keys}
        fl = max(1, out["route_flushes"])
        out["stage_ms_per_flush"] = {k[9:]: round((s1[k] - s0.get(k, 0)) / 1e3 / fl, 3) for k in s1
                                     if k.startswith("route_us_")}
        return out

    # ---- phases ------------------------------------------------------------------------------
    def single(self):
        st, sv, store = self.stack({})
        try:
            ctx = {"weather": "Sunny", "traffic": "Medium", "pickup_time": PICKUPS[0]}
            bodies = self.payloads(1000, lambda i: ctx, store)
            self.window(st, bodies, 64, 2.0)                     # context built, chains warm
            s0 = st.front.stats()
            w = self.window(st, bodies, self.a.concurrency, self.a.seconds)
            out = {"phase": "single", "contexts": 1, **w, **self.delta(st, s0)}
        finally:
            self.close(st, sv, store)
        self.single_p99 = out["p99_ms"]
        emit(out)
        return out

    def cycle64(self):
        st, sv, store = self.stack({})
        try:
            ctxs = [{"weather": w, "traffic": t, "pickup_time": p} for p in PICKUPS for w in WEATHERS
                    for t in TRAFFICS]
            bodies = self.payloads(1024, lambda i: ctxs[i % 64], store)
            s0 = st.front.stats()
            cold = self.window(st, bodies, self.a.concurrency, self.a.seconds)
            cold.update(self.delta(st, s0))
            s0 = st.front.stats()
            steady = self.window(st, bodies, self.a.concurrency, self.a.seconds)
            steady.update(self.delta(st, s0))
            stats = self.prov.router(self.dev).stats()
            out = {"phase": "cycle64", "contexts": 64, "cold": cold, "steady": steady,
                   "cache_capacity": stats.get("cache_capacity"), "async_built": stats.get("async_built")}
            sp = getattr(self, "single_p99", None)
            if sp:
                out["p99_vs_single"] = round(steady["p99_ms"] / sp, 3)
        finally:
            self.close(st, sv, store)
        emit(out)
        return out

    def hour(self, prefetch=True, extra_hours=0):
        # the route clock at hh:59:30 (+ extra_hours) when the stack is built; runs start 12 s
        # before the boundary
        lt = time.localtime()
        sec_in_hour = lt.tm_min * 60 + lt.tm_sec
        skew = (3600 - 30 - sec_in_hour) % 3600 + 3600 * extra_hours
        env = {"ROUTEST_ROUTE_CLOCK_SKEW_S": str(skew)}
        if not prefetch:
            env["ROUTEST_CCH_PREFETCH_MIN"] = "0"
        st, sv, store = self.stack(env)
        name = "hour" if prefetch else "hour_noprefetch"
        s_start = st.front.stats()
        try:
            bodies = self.payloads(1000, lambda i: None, store)        # F02 context: routed at "now"
            self.window(st, bodies, 64, 2.0)                           # the current hour built
            t_boundary = time.time() + (3600 - (int(time.time() + skew) % 3600))
            lead = t_boundary - time.time()
            if lead > 12:
                time.sleep(lead - 12)
            s0 = st.front.stats()
            wins = []
            for k in range(self.a.hour_windows):
                t_start = time.time()
                w = self.window(st, bodies, self.a.concurrency, 1.0)
                w["t_rel_boundary_s"] = round(t_start - t_boundary, 2)
                wins.append(w)
                emit({"phase": name, "window": k, **w})
            before = [w for w in wins if w["t_rel_boundary_s"] + w["s"] <= 0][1:] or wins[:1]
            after = [w for w in wins if w["t_rel_boundary_s"] + w["s"] > 0]
            steady_p99 = float(np.median([w["p99_ms"] for w in before]))
            out = {"phase": name, "prefetch": prefetch, "windows": len(wins),
                   "steady_p99_ms": steady_p99,
                   "max_ms_after_boundary": max(w["max_ms"] for w in after) if after else None,
                   "max_p99_ms_after_boundary": max(w["p99_ms"] for w in after) if after else None,
                   "errors": sum(w["errors"] for w in wins), **self.delta(st, s0),
                   "prefetched_since_start": st.front.stats().get("route_ctx_prefetched", 0)
                   - s_start.get("route_ctx_prefetched", 0)}
            if after:
                out["worst_after_vs_steady_p99"] = round(out["max_ms_after_boundary"] / steady_p99, 3)
        finally:
            self.close(st, sv, store)
        emit(out)
        return out

    def fresh(self):
        st, sv, store = self.stack({})
        try:
            ctx = {"weather": "Sunny", "traffic": "Medium", "pickup_time": PICKUPS[0]}
            bodies = self.payloads(1000, lambda i: ctx, store)
            for _ in range(30):                        # until the cached context is built and warm
                w = self.window(st, bodies, 64, 1.0)
                if w["requests"] > 0 and w["max_ms"] < 1000:
                    break
            fresh_ctx = [{"weather": w, "traffic": "Jam", "pickup_time": PICKUPS[3]} for w in WEATHERS]
            fresh_bodies = self.payloads(4, lambda i: fresh_ctx[i], store, seed=7)
            res = []

            def side():
                c = http.client.HTTPConnection("127.0.0.1", st.port, timeout=120)
                for b in fresh_bodies:
                    t0 = time.perf_counter()
                    c.request("POST", "/api/optimize_route", body=b.encode(),
                              headers={"Content-Type": "application/json"})
                    r = c.getresponse()
                    r.read()
                    res.append({"status": r.status, "ms": round((time.perf_counter() - t0) * 1e3, 2)})
            s0 = st.front.stats()
            wins, th = [], None
            for k in range(self.a.fresh_windows):
                if k == 4:
                    th = threading.Thread(target=side)
                    th.start()
                alive = th is not None and th.is_alive()
                sw = st.front.stats()
                w = self.window(st, bodies, self.a.concurrency, 0.5)
                w["stage_ms_per_flush"] = self.delta(st, sw)["stage_ms_per_flush"]
                w["fresh_in_flight"] = alive or (th is not None and th.is_alive())
                wins.append(w)
                emit({"phase": "fresh", "window": k, **w})
            th.join()
            base = wins[1:4]
            during = [w for w in wins[4:] if w["fresh_in_flight"]] or wins[4:5]
            stats = self.prov.router(self.dev).stats()
            out = {"phase": "fresh", "fresh_requests": res,
                   "cached_p99_before_ms": max(w["p99_ms"] for w in base),
                   "cached_max_before_ms": max(w["max_ms"] for w in base),
                   "cached_p99_during_ms": max(w["p99_ms"] for w in during),
                   "cached_max_during_ms": max(w["max_ms"] for w in during),
                   **{k: stats.get(k) for k in ("async_built", "async_build_ms", "async_alloc_ms",
                                                "async_hostcopy_ms", "builder_max_wg", "async_paced")},
                   **self.delta(st, s0)}
        finally:
            self.close(st, sv, store)
        emit(out)
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--concurrency", type=int, default=1000)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--hour-windows", type=int, default=24)
    ap.add_argument("--fresh-windows", type=int, default=12)
    ap.add_argument("--phases", default="single,cycle64,hour,hour_noprefetch")
    a = ap.parse_args()
    b = Bench(a)
    res = {}
    for ph in a.phases.split(","):
        if ph == "single":
            res[ph] = b.single()
        elif ph == "cycle64":
            res[ph] = b.cycle64()
        elif ph == "hour":
            res[ph] = b.hour(True)
        elif ph == "hour_noprefetch":
            res[ph] = b.hour(False, extra_hours=2)     # a boundary whose contexts are not cached
        elif ph == "fresh":
            res[ph] = b.fresh()
        else:
            raise SystemExit(f"unknown phase {ph}")
    summ = {"stage": "summary", "nodes": b.g.num_nodes, "concurrency": a.concurrency}
    if "cycle64" in res:
        summ["cycle64_p99_vs_single"] = res["cycle64"].get("p99_vs_single")
    for k in ("hour", "hour_noprefetch"):
        if k in res:
            summ[f"{k}_worst_after_vs_steady_p99"] = res[k].get("worst_after_vs_steady_p99")
    if "fresh" in res:
        f = res["fresh"]
        summ["fresh_cached_max_during_vs_before"] = round(f["cached_max_during_ms"] / f["cached_max_before_ms"], 3)
    emit(summ)


if __name__ == "__main__":
    main()
