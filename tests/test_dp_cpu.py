"""Data-parallel training logic on CPU with Gloo (world_size 2/4/8, torch.multiprocessing.spawn):
the flat-bucket all-reduce must give exactly the single-process large-batch gradient, all ranks
must end with identical weights, and checkpoints must resume."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from routest_amd.data.synth import synth_records
from routest_amd.models.features import records_to_features
from routest_amd.models.mlp3 import EtaMLP
from routest_amd.ops.eta_mlp import featurize_torch, records_to_tensor
from routest_amd.parallel.dp import FlatGrads, allreduce_flat, bucket_slices


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _model():
    torch.manual_seed(0)
    m = EtaMLP(64)
    rec, y = synth_records(4096, 0)
    m.fit_normalization(records_to_features(rec), y)
    return m


def _grad_worker(rank, world, port, out_dir):
    _setup(rank, world, port)
    m = _model()
    rec, y = synth_records(256 * world, 5)
    rec = records_to_tensor(rec)
    y = (torch.from_numpy(y) - m.y_mean) / m.y_std
    fg = FlatGrads(list(m.parameters()))
    sl = slice(rank * 256, (rank + 1) * 256)
    loss = torch.nn.functional.mse_loss(m.forward_normalized(featurize_torch(rec[sl])), y[sl])
    loss.backward()
    fg.allreduce_avg()
    torch.save(fg.buf.clone(), os.path.join(out_dir, f"g{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_gradient_equals_large_batch(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_grad_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        gs = [torch.load(os.path.join(d, f"g{r}.pt")) for r in range(world)]
    for g in gs[1:]:
        assert torch.equal(g, gs[0])
    m = _model()
    rec, y = synth_records(256 * world, 5)
    y = (torch.from_numpy(y) - m.y_mean) / m.y_std
    fg = FlatGrads(list(m.parameters()))
    torch.nn.functional.mse_loss(m.forward_normalized(featurize_torch(records_to_tensor(rec))), y).backward()
    torch.testing.assert_close(gs[0], fg.buf, rtol=1e-5, atol=1e-7)


def _train_worker(rank, world, port, out_dir, steps, ckpt):
    _setup(rank, world, port)
    from routest_amd.train.trainer import TrainConfig, Trainer
    cfg = TrainConfig(hidden=64, batch_local=512, steps=steps, rows_per_rank=4096, log_every=10,
                      eval_rows=1024, ckpt_dir=ckpt, warmup=5, dist_backend="gloo")
    tr = Trainer(cfg)
    res = tr.fit()
    from routest_amd.train.fused import flatten_params
    torch.save({"p": flatten_params(tr.model), "res": res}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_dp_training_ranks_in_sync_and_resume():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        ck = os.path.join(d, "ckpt")
        mp.spawn(_train_worker, args=(world, _free_port(), d, 30, ck), nprocs=world, join=True)
        r0 = torch.load(os.path.join(d, "r0.pt"), weights_only=False)
        r1 = torch.load(os.path.join(d, "r1.pt"), weights_only=False)
        assert torch.equal(r0["p"], r1["p"])
        h = r0["res"]["history"]
        assert h[-1]["mse_norm"] < 1.0
        from routest_amd.models.checkpoint import resolve_checkpoint
        assert os.path.exists(os.path.join(resolve_checkpoint(ck), "optimizer.safetensors"))
        # resume: continues from step 30 for 10 more steps
        mp.spawn(_train_worker, args=(world, _free_port(), d, 10, ck), nprocs=world, join=True)
        r0b = torch.load(os.path.join(d, "r0.pt"), weights_only=False)
        assert r0b["res"]["history"][-1]["step"] == 40
        assert not torch.equal(r0b["p"], r0["p"])


def test_allreduce_flat_single_process_noop():
    b = torch.arange(5.0)
    assert torch.equal(allreduce_flat(b.clone()), b)


def test_bucket_slices():
    s = bucket_slices(10, bucket_bytes=16)
    assert s == [(0, 4), (4, 8), (8, 10)]
    assert bucket_slices(69904) == [(0, 69904)]
