"""ETA model training entrypoint (configs 1-3) — the "notebook training entrypoint" the reference
README lists as "Coming Soon" (``README.md:13-18``; ``notebooks/.gitkeep``).

* ``arch=linear``: closed-form least squares on a CSV (config 1, CPU).
* ``arch=mlp3``  : data-parallel AdamW training, one process per GPU under ``torchrun``.
  Backend ``fused`` (default on GPUs) = the HIP kernels of :mod:`train.fused`; backend
  ``autograd`` = plain PyTorch (CPU / Gloo CI and the numerical reference).  Both reduce ONE flat
  gradient bucket per step and produce identical checkpoints (``models/checkpoint.py``).

Resume: if ``ckpt_dir`` holds a checkpoint with ``trainer_state.json`` the run continues from its
step with the saved optimizer moments (``torchrun --max-restarts`` relaunches land here).
"""
from __future__ import annotations

import json
import os
import time
from dataclasses import asdict, dataclass
from typing import Any, Dict, Optional

import numpy as np
import torch

from ..data.synth import read_trips_csv, synth_records, synth_trips
from ..models.checkpoint import checkpoint_exists, load_checkpoint, load_training_state, save_checkpoint
from ..models.features import features_to_records, records_to_features
from ..models.mlp3 import EtaMLP, LinearETA
from ..ops.eta_mlp import featurize_torch, records_to_tensor
from ..parallel.dp import DistInfo, FlatGrads, allreduce_scalars, barrier, broadcast_flat, init_distributed
from ..utils.faults import fault_step
from ..utils.logging import get_logger
from .fused import FusedMlp3Trainer, flatten_params, lr_at, unflatten_into

log = get_logger("train")


@dataclass
class TrainConfig:
    arch: str = "mlp3"
    hidden: int = 256
    batch_local: int = 65536
    steps: int = 500
    lr: float = 2e-3
    weight_decay: float = 0.0
    warmup: int = 20
    min_lr_ratio: float = 0.1
    rows_per_rank: int = 1 << 20
    data_csv: str = ""
    seed: int = 0
    backend: str = "auto"          # auto | fused | autograd
    log_every: int = 50
    log_path: str = ""
    ckpt_dir: str = ""
    ckpt_every: int = 0
    eval_rows: int = 65536
    dist_backend: str = ""         # "" = nccl on GPU, gloo on CPU
    comm: str = "torch"            # gradient all-reduce: torch (ProcessGroup) | rccl | oneshot (native, fused backend)
    max_steps: int = 0             # > 0: train until this ABSOLUTE step (elastic relaunches resume and stop here)


def train_linear(cfg: TrainConfig) -> LinearETA:
    if cfg.data_csv:
        x, y = read_trips_csv(cfg.data_csv)
    else:
        x, y = synth_trips(1000, cfg.seed)
    m = LinearETA().fit(x, y)
    if cfg.ckpt_dir:
        save_checkpoint(cfg.ckpt_dir, m, trainer_state={"step": 0, "config": asdict(cfg)})
    return m


class Trainer:
    def __init__(self, cfg: TrainConfig, dist_info: Optional[DistInfo] = None):
        self.cfg = cfg
        self.di = dist_info or init_distributed(cfg.dist_backend or None)
        dev = self.di.device
        self.backend = cfg.backend
        if self.backend == "auto":
            self.backend = "fused" if dev.type == "cuda" else "autograd"
        torch.manual_seed(cfg.seed)
        np.random.seed(cfg.seed + self.di.rank)
        self.start_step = 0
        resumed = self._maybe_resume()
        if not resumed:
            self.model = EtaMLP(cfg.hidden)
            # normalisation statistics from a fixed synthetic sample: identical on every rank
            xs, ys = synth_trips(65536, seed=12345)
            self.model.fit_normalization(xs, ys)
            flat = flatten_params(self.model).to(dev)
            broadcast_flat(flat, 0)
            unflatten_into(self.model, flat)
        self.global_batch = cfg.batch_local * self.di.world
        self._load_data()
        self._setup_backend()
        self.history: list = []

    # ---------------------------------------------------------------- data
    def _load_data(self) -> None:
        cfg, dev = self.cfg, self.di.device
        if cfg.data_csv:
            x, y = read_trips_csv(cfg.data_csv)
            shard = slice(self.di.rank, None, self.di.world)
            rec = features_to_records(x[shard])
            y = y[shard]
        else:
            rec, y = synth_records(cfg.rows_per_rank, seed=1000 + cfg.seed * 97 + self.di.rank)
        n = (len(y) // cfg.batch_local) * cfg.batch_local
        if n == 0:
            reps = -(-cfg.batch_local // len(y))
            rec = np.tile(rec, reps)[:cfg.batch_local]
            y = np.tile(y, reps)[:cfg.batch_local]
            n = cfg.batch_local
        self.rec = records_to_tensor(rec[:n]).to(dev)
        y_t = torch.from_numpy(np.asarray(y[:n], dtype=np.float32)).to(dev)
        self.y_raw = y_t
        self.y_norm = ((y_t - float(self.model.y_mean)) / float(self.model.y_std)).contiguous()
        self.nbatches = n // cfg.batch_local
        erec, ey = synth_records(cfg.eval_rows, seed=777)
        self.eval_rec = records_to_tensor(erec).to(dev)
        self.eval_y = torch.from_numpy(ey).to(dev)

    def batch(self, step: int):
        b = step % self.nbatches
        s = b * self.cfg.batch_local
        e = s + self.cfg.batch_local
        return self.rec[s:e], self.y_norm[s:e]

    # ---------------------------------------------------------------- backends
    def _setup_backend(self) -> None:
        cfg = self.cfg
        total = cfg.max_steps if cfg.max_steps > 0 else self.start_step + cfg.steps
        if self.backend == "fused":
            self.fused = FusedMlp3Trainer(self.model, self.di.device, cfg.batch_local, self.global_batch,
                                          lr=cfg.lr, weight_decay=cfg.weight_decay, warmup=cfg.warmup,
                                          total_steps=total, min_lr_ratio=cfg.min_lr_ratio,
                                          allreduce=self.di.world > 1, comm=self._native_comm())
            if self._opt_state is not None:
                self.fused.load_optimizer_state(self._opt_state)
        else:
            self.model = self.model.to(self.di.device)
            self.flat = FlatGrads(list(self.model.parameters()))
            wd_params = [self.model.l1.weight, self.model.l2.weight, self.model.l3.weight]
            nd_params = [self.model.l1.bias, self.model.l2.bias, self.model.l3.bias]
            self.opt = torch.optim.AdamW([{"params": wd_params, "weight_decay": cfg.weight_decay},
                                          {"params": nd_params, "weight_decay": 0.0}],
                                         lr=cfg.lr, betas=(0.9, 0.999), eps=1e-8)
            self.sched = torch.optim.lr_scheduler.LambdaLR(
                self.opt, lambda k: lr_at(k + 1, 1.0, cfg.warmup, total, cfg.min_lr_ratio))
            if self._opt_state is not None:
                self._load_torch_opt(self._opt_state)

    def _native_comm(self):
        if self.cfg.comm == "torch" or self.di.world == 1:
            return None
        from ..parallel.comm import DeviceComm
        c = DeviceComm(self.di.device)
        if self.cfg.comm == "oneshot" and not c.oneshot:
            raise RuntimeError("one-shot all-reduce needs all ranks on one node (<= 8 GPUs)")
        return c

    def _load_torch_opt(self, st: Dict[str, torch.Tensor]) -> None:
        m_flat, v_flat = st["exp_avg"], st["exp_avg_sq"]
        step = int(st["step"].reshape(-1)[0])
        order = [self.model.l1.weight, self.model.l1.bias, self.model.l2.weight, self.model.l2.bias,
                 self.model.l3.weight, self.model.l3.bias]
        o = 0
        for p in order:
            n = p.numel()
            self.opt.state[p] = {"step": torch.tensor(float(step)),
                                 "exp_avg": m_flat[o:o + n].view_as(p).to(p.device).clone(),
                                 "exp_avg_sq": v_flat[o:o + n].view_as(p).to(p.device).clone()}
            o += n
        self.sched.last_epoch = step
        for g in self.opt.param_groups:
            g["lr"] = self.cfg.lr * lr_at(step + 1, 1.0, self.cfg.warmup, self.start_step + self.cfg.steps,
                                          self.cfg.min_lr_ratio)

    def _torch_opt_flat(self) -> Dict[str, torch.Tensor]:
        order = [self.model.l1.weight, self.model.l1.bias, self.model.l2.weight, self.model.l2.bias,
                 self.model.l3.weight, self.model.l3.bias]
        ms, vs, step = [], [], 0
        for p in order:
            st = self.opt.state.get(p, {})
            ms.append(st.get("exp_avg", torch.zeros_like(p)).detach().reshape(-1).cpu())
            vs.append(st.get("exp_avg_sq", torch.zeros_like(p)).detach().reshape(-1).cpu())
            step = int(st.get("step", torch.tensor(0.0)).item()) if st else step
        return {"exp_avg": torch.cat(ms), "exp_avg_sq": torch.cat(vs), "step": torch.tensor([step])}

    # ---------------------------------------------------------------- resume / ckpt
    def _maybe_resume(self) -> bool:
        self._opt_state = None
        d = self.cfg.ckpt_dir
        if not checkpoint_exists(d):
            return False
        model, _ = load_checkpoint(d)
        opt, ts = load_training_state(d)
        self.model = model
        self._opt_state = opt
        self.start_step = int((ts or {}).get("step", 0))
        log.info("resumed from %s at step %d", d, self.start_step)
        return True

    def save(self, step: int) -> None:
        if not self.cfg.ckpt_dir or not self.di.is_main:
            return
        if self.backend == "fused":
            model = self.fused.to_model()
            opt = self.fused.optimizer_state()
        else:
            model = self.model
            opt = self._torch_opt_flat()
        save_checkpoint(self.cfg.ckpt_dir, model, optimizer_state=opt,
                        trainer_state={"step": step, "config": asdict(self.cfg), "world": self.di.world})

    # ---------------------------------------------------------------- loop
    def train_step(self, step: int) -> Optional[torch.Tensor]:
        rec, y = self.batch(step)
        if self.backend == "fused":
            return self.fused.step(rec, y)
        self.flat.zero()
        pred = self.model.forward_normalized(featurize_torch(rec))
        loss = torch.nn.functional.mse_loss(pred, y)
        loss.backward()
        self.flat.allreduce_avg()
        self.opt.step()
        self.sched.step()
        return loss.detach().reshape(1) * self.cfg.batch_local

    def evaluate(self) -> Dict[str, float]:
        from ..ops.eta_mlp import EtaMlpKernel
        model = self.fused.to_model() if self.backend == "fused" else self.model
        with torch.no_grad():
            if self.di.device.type == "cuda" and model.hidden in (64, 128, 256):
                pred = EtaMlpKernel(model, self.di.device)(self.eval_rec)
            else:
                pred = model.to(self.di.device)(featurize_torch(self.eval_rec))
        err = pred.float() - self.eval_y
        return {"mae_min": float(err.abs().mean()), "rmse_min": float(err.pow(2).mean().sqrt())}

    def fit(self) -> Dict[str, Any]:
        cfg = self.cfg
        dev = self.di.device
        logf = open(cfg.log_path, "a") if (cfg.log_path and self.di.is_main) else None
        t0 = time.perf_counter()
        last_t, last_s = t0, self.start_step
        end = cfg.max_steps if cfg.max_steps > 0 else self.start_step + cfg.steps
        crash_at = fault_step("rank_crash")
        first_attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") == "0"
        for step in range(self.start_step, end):
            lt = self.train_step(step)
            s1 = step + 1
            if crash_at == s1 and first_attempt and self.di.rank == self.di.world - 1:
                log.error("injected fault: rank %d exits hard at step %d", self.di.rank, s1)
                os._exit(13)
            if (cfg.log_every and s1 % cfg.log_every == 0) or s1 == end:
                loss_sum = float(lt.sum().item())
                tot = allreduce_scalars([loss_sum], dev)[0] / self.global_batch
                now = time.perf_counter()
                rate = (s1 - last_s) * self.global_batch / max(1e-9, now - last_t)
                last_t, last_s = now, s1
                rec = {"step": s1, "mse_norm": tot, "samples_per_s": rate,
                       "lr": lr_at(s1, cfg.lr, cfg.warmup, end, cfg.min_lr_ratio)}
                self.history.append(rec)
                if logf:
                    logf.write(json.dumps(rec) + "\n")
                    logf.flush()
            if cfg.ckpt_every and s1 % cfg.ckpt_every == 0:
                barrier(dev)
                self.save(s1)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        self.save(end)
        ev = self.evaluate()
        out = {"steps": end - self.start_step, "start_step": self.start_step, "end_step": end, "wall_s": wall, "global_batch": self.global_batch,
               "samples_per_s": (end - self.start_step) * self.global_batch / wall, "world": self.di.world,
               "backend": self.backend, **ev, "history": self.history[-3:]}
        if logf:
            logf.write(json.dumps({k: v for k, v in out.items() if k != "history"}) + "\n")
            logf.close()
        return out


def main(argv=None) -> None:
    import argparse
    ap = argparse.ArgumentParser(description="Train the routest_amd ETA model (torchrun for >1 GPU)")
    for f, v in asdict(TrainConfig()).items():
        ap.add_argument("--" + f.replace("_", "-"), type=type(v), default=v)
    a = ap.parse_args(argv)
    cfg = TrainConfig(**{k.replace("-", "_"): v for k, v in vars(a).items()})
    if cfg.arch == "linear":
        m = train_linear(cfg)
        print(json.dumps({"arch": "linear", "coef": m.coef.tolist(), "intercept": m.intercept}))
        return
    tr = Trainer(cfg)
    res = tr.fit()
    if tr.di.is_main:
        print(json.dumps(res))
    from ..parallel.dp import shutdown
    shutdown()


if __name__ == "__main__":
    main()
