"""``python -m routest_amd <command>`` — serve | train | bench | export | synth.

Config is loaded (``.env`` first, then the environment, then flags) BEFORE any service module
reads it — the reference imports its route modules before ``load_dotenv()`` runs, so `.env`-only
settings never reached them (``RO/app.py:1-4``).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys


def cmd_serve(a: argparse.Namespace) -> None:
    from .config import load_settings, set_settings
    over = {}
    if a.device:
        over["device"] = a.device
    if a.provider:
        over["provider"] = a.provider
    if a.store:
        over["store_url"] = a.store
    if a.graph:
        over["graph_path"] = a.graph
        over.setdefault("provider", "graph")
    s = load_settings(dotenv_path=a.env_file, **over)
    set_settings(s)
    from .utils.logging import setup_logging
    setup_logging(s.log_json)
    from .api.app import build_services, create_app
    from .serve.eta_service import EtaService, default_model
    eta = None
    if a.synthetic_model:
        eta = EtaService(default_model(hidden=a.hidden), device=s.device, devices=s.devices,
                         batch_max=s.batch_max, timeout_us=s.batch_timeout_us)
    elif a.model:
        eta = EtaService(model_path=a.model, device=s.device, devices=s.devices, batch_max=s.batch_max,
                         timeout_us=s.batch_timeout_us, allow_pickle=os.environ.get("ROUTEST_ALLOW_PICKLE") == "1")
    sv = build_services(s, eta=eta)
    app = create_app(sv)
    port = a.port or s.port
    from .serve.native_server import native_supported
    native_ok = eta is not None and eta.backend == "hip" and bool(eta.devices) and native_supported(eta.model)
    if a.front == "native" and native_ok:
        # the native front end owns the main port; the FastAPI app answers what it relays
        from .serve.frontend import ServingStack
        stack = ServingStack(sv, app, eta.model, [d.index for d in eta.devices], port=port,
                             threads=a.native_threads, bind_any=a.host not in ("127.0.0.1", "localhost"))
        print(json.dumps({"port": stack.port, "front": "native", "app_port": stack.app_server.port,
                          "native_routes": bool(stack.front.routes)}), flush=True)
        import threading
        try:
            threading.Event().wait()
        except KeyboardInterrupt:
            pass
        finally:
            stack.close()
        return
    native_srv = None
    if a.native_port and native_ok:
        from .serve.native_server import NativePredictServer
        native_srv = NativePredictServer(eta.model, device=[d.index for d in eta.devices], port=a.native_port,
                                         threads=a.native_threads, cors_origins=s.cors_origins,
                                         bind_any=a.host not in ("127.0.0.1", "localhost"))
        print(json.dumps({"native_predict_port": native_srv.port}), flush=True)
    import uvicorn
    try:
        uvicorn.run(app, host=a.host, port=port, log_level="warning", access_log=False)
    finally:
        if native_srv is not None:
            native_srv.close()


def cmd_train(a: argparse.Namespace, rest) -> None:
    from .train.trainer import main as train_main
    train_main(rest)


def cmd_bench(a: argparse.Namespace, rest) -> None:
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = {"serve": "bench.py", "train": "bench/train_bench.py", "gcn": "bench/gcn_bench.py",
              "route": "bench/route_bench.py", "rccl": "bench/rccl_bench.py", "http": "bench/http_bench.py",
              "kernel": "bench/eta_kernel_sweep.py"}[a.what]
    cmd = [sys.executable, os.path.join(root, script)] + list(rest)
    if a.nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--nproc-per-node", str(a.nproc),
               os.path.join(root, script)] + list(rest)
    raise SystemExit(subprocess.call(cmd))


def cmd_export(a: argparse.Namespace) -> None:
    from .models.checkpoint import export_predictor_pickle, load_checkpoint
    model, _ = load_checkpoint(a.checkpoint)
    export_predictor_pickle(model, a.out)
    print(json.dumps({"exported": a.out, "arch": model.arch}))


def cmd_synth(a: argparse.Namespace) -> None:
    from .data.synth import write_trips_csv
    write_trips_csv(a.out, a.rows, a.seed)
    print(json.dumps({"csv": a.out, "rows": a.rows}))


def main(argv=None) -> None:
    from .utils.profiling import apply_debug_env
    apply_debug_env()          # ROUTEST_DEBUG_SYNC=1: serialised kernels, synchronous launch errors
    ap = argparse.ArgumentParser(prog="routest_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("serve", help="run the HTTP API (uvicorn)")
    s.add_argument("--host", default="127.0.0.1")
    s.add_argument("--port", type=int, default=0)
    s.add_argument("--model", default="", help="checkpoint dir | XGBoost JSON | pickle (opt-in)")
    s.add_argument("--synthetic-model", action="store_true", help="train a small MLP on synthetic trips")
    s.add_argument("--hidden", type=int, default=256)
    s.add_argument("--device", default="")
    s.add_argument("--provider", default="")
    s.add_argument("--graph", default="", help="road graph file for --provider graph (.gr+.co DIMACS, "
                   ".edges.csv+.nodes.csv, .npz); default: the synthetic Metro-Manila graph")
    s.add_argument("--store", default="")
    s.add_argument("--env-file", default=".env")
    s.add_argument("--front", choices=["native", "python"], default="native",
                   help="native: the C++ front end owns the main port (predictions and routes natively, "
                        "everything else relayed to the FastAPI app); python: uvicorn on the main port")
    s.add_argument("--native-port", type=int, default=0,
                   help="(--front python) also serve /api/predict_eta and /predict natively on this port")
    s.add_argument("--native-threads", type=int, default=8)
    t = sub.add_parser("train", help="train the ETA model (use torchrun for multi-GPU)")
    b = sub.add_parser("bench", help="run a benchmark")
    b.add_argument("what", choices=["serve", "train", "gcn", "route", "rccl", "http", "kernel"])
    b.add_argument("--nproc", type=int, default=1)
    e = sub.add_parser("export", help="checkpoint -> picklable EtaPredictor for the reference loader")
    e.add_argument("checkpoint")
    e.add_argument("out")
    y = sub.add_parser("synth", help="write the config-1 synthetic trip CSV")
    y.add_argument("out")
    y.add_argument("--rows", type=int, default=1000)
    y.add_argument("--seed", type=int, default=0)
    a, rest = ap.parse_known_args(argv)
    if a.cmd == "serve":
        cmd_serve(a)
    elif a.cmd == "train":
        cmd_train(a, rest)
    elif a.cmd == "bench":
        cmd_bench(a, rest)
    elif a.cmd == "export":
        cmd_export(a)
    elif a.cmd == "synth":
        cmd_synth(a)


if __name__ == "__main__":
    main()
