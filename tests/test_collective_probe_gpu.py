"""The collective sweep bench.py runs after its timed region on multi-GPU nodes
(parallel/collective_probe.py): exercised here on a 1-rank RCCL group (the driver's 8-GPU runs are
the only place it sees real xGMI peers)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_sweep_single_rank_rccl():
    import torch.distributed as dist
    from routest_amd.parallel.collective_probe import sweep
    from routest_amd.parallel.launch import free_port
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        rows = sweep(dev, sizes=(296_000, 4 << 20))
    finally:
        dist.destroy_process_group()
    ops = {(r["op"], r["bytes"]) for r in rows}
    assert ("all_reduce", 296_000) in ops and any(o == "all_gather" for o, _ in ops)
    assert all(r["us"] > 0 and r["busbw_GBps"] == 0.0 for r in rows)   # n = 1: nothing crosses a link
