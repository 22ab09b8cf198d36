"""The keys of ``bench.py``'s JSON line, in ONE place.

``bench.py`` builds every section through the builders below and appends ``schema_problems`` (the
output of :func:`problems`, empty when the line is complete) before it prints; the GPU tests
(``tests/test_multigpu.py``, ``tests/test_bench_contract_gpu.py``) read keys through the constants
here, and ``tests/test_bench_schema_cpu.py`` runs the builders and the rank reductions on the CPU
(gloo, 2 ranks) — so a renamed key fails on the CPU, not in the driver's first 8-GPU run.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

#: the driver's contract (task statement; BASELINE.json metric/config)
HEADLINE = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config")
CONFIG = ("model", "global_batch", "seq_len", "parallelism")
#: extra top-level sections (present, possibly null when skipped by flags)
SECTIONS = ("collectives", "dp_training", "dp_training_oneshot", "dp_training_large_batch", "gcn",
            "route_optimizer", "shared_gpu", "finite", "schema_problems")

DP_TRAINING = ("samples_per_s", "ms_per_step", "batch_per_gpu", "global_batch", "steps", "allreduce",
               "final_local_mse_normalized")
DP_ONESHOT_EXTRA = ("comm_error", "params_identical_across_ranks")
GCN = ("nodes", "edges", "routes_per_step", "modes")
GCN_MODE = ("ms_per_step", "routes_per_s")
#: GCN modes by world size / comm availability (bench.py runs exactly these)
GCN_MODES_1 = ("replicate",)
GCN_MODES_N = ("replicate", "partition")
GCN_MODE_ONESHOT = "partition_oneshot"
ROUTE = ("requests_per_step", "steps", "engine", "ms_per_step", "requests_per_s", "legs_per_s",
         "unfound_legs", "graph_nodes", "context_customize_ms", "context_cost_ms",
         "context_customize_gpu_ms", "topology_build_s", "cch", "ranks")
ROUTE_UNFOUND = "unfound_legs"
#: route_optimizer.http* (native main port load, rank 0)
ROUTE_HTTP = ("concurrency", "seconds", "requests", "req_per_s", "p50_ms", "p99_ms", "errors",
              "stage_ms_per_flush")


def dp_training(samples_per_s: float, ms_per_step: float, batch_per_gpu: int, world: int, steps: int,
                allreduce: str, loss: float, **extra) -> Dict[str, Any]:
    d = {"samples_per_s": samples_per_s, "ms_per_step": ms_per_step, "batch_per_gpu": batch_per_gpu,
         "global_batch": batch_per_gpu * world, "steps": steps, "allreduce": allreduce,
         "final_local_mse_normalized": loss}
    d.update(extra)
    return d


def gcn_section(nodes: int, edges: int, routes_per_step: int) -> Dict[str, Any]:
    return {"nodes": nodes, "edges": edges, "routes_per_step": routes_per_step, "modes": []}


def gcn_mode(sec: Dict[str, Any], mode: str, seconds: float, steps: int, routes: int) -> None:
    sec[mode] = {"ms_per_step": seconds / steps * 1e3, "routes_per_s": routes * steps / seconds}
    sec["modes"].append(mode)


def route_section(requests_per_step: int, steps: int, seconds: float, legs: int, unfound: int,
                  graph_nodes: int, ctx_ms: float, ctx_info: Dict[str, Any], topo_s: float,
                  cch_stats: Dict[str, Any], ranks: int) -> Dict[str, Any]:
    return {"requests_per_step": requests_per_step, "steps": steps, "engine": "cch",
            "ms_per_step": seconds / steps * 1e3,
            "requests_per_s": requests_per_step * steps / seconds,
            "legs_per_s": legs / seconds, "unfound_legs": unfound,
            "graph_nodes": graph_nodes,
            "context_customize_ms": ctx_ms,
            "context_cost_ms": ctx_info.get("cost_ms"),
            "context_customize_gpu_ms": ctx_info.get("customize_ms"),
            "topology_build_s": topo_s,
            "cch": dict(cch_stats), "ranks": ranks}


def reduce_route_stats(seconds: float, legs: int, unfound: int, device=None):
    """The route section's cross-rank reduction: the slowest rank's time (MAX) and the legs /
    unfound legs of all ranks (SUM).  CPU tensors under gloo (the shared-GPU rehearsal and the CPU
    test), device tensors under RCCL."""
    from ..parallel.dp import allreduce_scalars
    (t,) = allreduce_scalars([seconds], device, "max")
    lg, uf = allreduce_scalars([float(legs), float(unfound)], device, "sum")
    return t, int(lg), int(uf)


def _missing(d: Optional[Dict[str, Any]], keys: Sequence[str], where: str) -> List[str]:
    if d is None:
        return []
    if not isinstance(d, dict):
        return [f"{where}: not an object"]
    if "error" in d:
        return [f"{where}: error {str(d['error'])[:120]}"]
    return [f"{where}.{k}" for k in keys if k not in d]


def problems(d: Dict[str, Any]) -> List[str]:
    """Missing keys / section errors of a bench line ([] when complete).  Skipped sections are
    ``None`` and pass; a section that ran must carry every key."""
    out = [k for k in HEADLINE + SECTIONS if k not in d and k != "schema_problems"]
    out += _missing(d.get("config"), CONFIG, "config")
    out += _missing(d.get("dp_training"), DP_TRAINING, "dp_training")
    out += _missing(d.get("dp_training_large_batch"), DP_TRAINING, "dp_training_large_batch")
    out += _missing(d.get("dp_training_oneshot"), DP_TRAINING + DP_ONESHOT_EXTRA, "dp_training_oneshot")
    g = d.get("gcn")
    out += _missing(g, GCN, "gcn")
    if isinstance(g, dict) and "error" not in g:
        for m in g.get("modes", []):
            out += _missing(g.get(m), GCN_MODE, f"gcn.{m}")
    r = d.get("route_optimizer")
    out += _missing(r, ROUTE, "route_optimizer")
    if isinstance(r, dict) and "error" not in r:
        for k in ("http", "http_f02"):
            if k in r:
                out += _missing(r[k], ROUTE_HTTP, f"route_optimizer.{k}")
    if d.get("serving_error"):
        out.append(f"serving: error {str(d['serving_error'])[:120]}")
    coll = d.get("collectives")
    if isinstance(coll, list) and coll and isinstance(coll[0], dict) and "error" in coll[0]:
        out.append(f"collectives: error {str(coll[0]['error'])[:120]}")
    return out
