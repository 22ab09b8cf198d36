"""K3 training kernels on the GPU vs PyTorch fp32 autograd references."""
import copy

import pytest
import torch

from routest_amd.data.synth import synth_records
from routest_amd.models.features import records_to_features
from routest_amd.models.mlp3 import EtaMLP
from routest_amd.ops.eta_mlp import featurize_torch, pack_mlp3, records_to_tensor
from routest_amd.train.fused import (FusedMlp3Trainer, flatten_params, grads_from_bucket,
                                    pack_train_blob)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _model(H, seed=0):
    torch.manual_seed(seed)
    m = EtaMLP(H)
    rec, y = synth_records(8192, seed)
    m.fit_normalization(records_to_features(rec), y)
    return m


def _batch(B, m, seed=3):
    rec, y = synth_records(B, seed)
    rt = records_to_tensor(rec)
    yn = (torch.from_numpy(y) - m.y_mean) / m.y_std
    return rt, yn.float()


@pytest.mark.parametrize("H", [64, 128, 256])
def test_initial_pack_matches_host_pack(H):
    m = _model(H)
    tr = FusedMlp3Trainer(m, DEV, 1024, 1024)
    mm = copy.deepcopy(m)
    mm.y_mean.fill_(0.0)
    mm.y_std.fill_(1.0)
    ref = pack_train_blob(mm)
    assert torch.equal(tr.blob.cpu(), ref)


@pytest.mark.parametrize("H", [64, 128, 256])
@pytest.mark.parametrize("B", [1000, 8192, 70000])
def test_fused_gradients_match_autograd(H, B):
    m = _model(H)
    rt, yn = _batch(B, m)
    tr = FusedMlp3Trainer(m, DEV, B, B)
    tr.forward_backward(rt.to(DEV), yn.to(DEV))
    torch.cuda.synchronize()
    got = grads_from_bucket(tr.G, H)
    ref_m = copy.deepcopy(m)
    loss = torch.nn.functional.mse_loss(ref_m.forward_normalized(featurize_torch(rt)), yn)
    loss.backward()
    for name, p in ref_m.named_parameters():
        g, r = got[name].reshape(-1), p.grad.reshape(-1)
        rel = (g - r).norm() / r.norm().clamp_min(1e-12)
        assert rel < 3e-2, (name, float(rel))
    # loss partials: per-tile squared errors of the forward pass
    mse = float(tr.loss_tiles.sum()) / B
    assert abs(mse - float(loss)) / float(loss) < 2e-2


def test_adamw_step_matches_torch():
    H, B = 64, 2048
    m = _model(H)
    rt, yn = _batch(B, m)
    tr = FusedMlp3Trainer(m, DEV, B, B, lr=1e-3, weight_decay=0.01)
    tr.forward_backward(rt.to(DEV), yn.to(DEV))
    g = grads_from_bucket(tr.G, H)
    p0 = flatten_params(m)
    tr.step_ctr.fill_(1)  # forward_backward already bumped it; one optimizer step = t=1
    tr._pack(update=True)
    torch.cuda.synchronize()
    ref = copy.deepcopy(m)
    for n, p in ref.named_parameters():
        p.grad = g[n].view_as(p).clone()
    opt = torch.optim.AdamW([{"params": [ref.l1.weight, ref.l2.weight, ref.l3.weight], "weight_decay": 0.01},
                             {"params": [ref.l1.bias, ref.l2.bias, ref.l3.bias], "weight_decay": 0.0}],
                            lr=1e-3, betas=(0.9, 0.999), eps=1e-8)
    opt.step()
    torch.testing.assert_close(tr.P.cpu(), flatten_params(ref), rtol=1e-5, atol=1e-6)
    assert not torch.equal(tr.P.cpu(), p0)


def _autograd_reference_train(m, rt, yn, B, steps, lr, warmup):
    """fp32 PyTorch autograd + torch AdamW with the fused trainer's schedule (lr_at)."""
    from routest_amd.train.fused import lr_at
    ref = copy.deepcopy(m).to(DEV)
    X = featurize_torch(rt)
    opt = torch.optim.AdamW(ref.parameters(), lr=lr, weight_decay=0.0)
    for s_ in range(steps):
        for g in opt.param_groups:
            g["lr"] = lr_at(s_ + 1, lr, warmup, steps, 0.1)
        k = s_ % 8
        loss = torch.nn.functional.mse_loss(ref.forward_normalized(X[k * B:(k + 1) * B]),
                                            yn[k * B:(k + 1) * B])
        opt.zero_grad()
        loss.backward()
        opt.step()
    return ref.cpu()


def test_fused_training_converges_and_serves():
    """The fused bf16 trainer reaches the accuracy of an fp32 autograd run with the same data,
    schedule and initialisation (error measured against the noise-free ground truth; the 5 %
    multiplicative label noise puts the floor at ~4 % MAE)."""
    from routest_amd.data.synth import eta_ground_truth
    from routest_amd.ops.eta_mlp import EtaMlpKernel
    H, B, steps = 128, 16384, 300
    m = _model(H, 1)
    rec, y = synth_records(B * 8, 11)
    rt = records_to_tensor(rec).to(DEV)
    yn = ((torch.from_numpy(y) - m.y_mean) / m.y_std).float().to(DEV)
    tr = FusedMlp3Trainer(copy.deepcopy(m), DEV, B, B, lr=3e-3, warmup=10, total_steps=steps)
    losses = []
    for s in range(steps):
        k = s % 8
        tr.step(rt[k * B:(k + 1) * B], yn[k * B:(k + 1) * B])
        if s % 50 == 0 or s == steps - 1:
            losses.append(tr.local_mse())
    assert losses[-1] < 0.2 * losses[0], losses
    model = tr.to_model()
    ref = _autograd_reference_train(m, rt, yn, B, steps, 3e-3, 10)
    erec, _ = synth_records(4096, 99)
    truth = torch.from_numpy(eta_ground_truth(records_to_features(erec)))
    pred = EtaMlpKernel(model, DEV)(records_to_tensor(erec).to(DEV)).cpu()
    with torch.no_grad():
        pref = ref(torch.from_numpy(records_to_features(erec))).reshape(-1)
    mae = float((pred - truth).abs().mean() / truth.mean())
    mae_ref = float((pref - truth).abs().mean() / truth.mean())
    assert mae < 0.12, (mae, mae_ref)
    assert mae <= 1.3 * mae_ref + 0.005, (mae, mae_ref)


def test_graph_captured_step_matches_eager():
    H, B = 64, 4096
    m = _model(H, 2)
    rt, yn = _batch(B, m, 4)
    rt, yn = rt.to(DEV), yn.to(DEV)
    eager = FusedMlp3Trainer(copy.deepcopy(m), DEV, B, B, lr=1e-3)
    graphed = FusedMlp3Trainer(copy.deepcopy(m), DEV, B, B, lr=1e-3)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm up hipBLASLt outside capture
        graphed.forward_backward(rt, yn)
    torch.cuda.current_stream().wait_stream(s)
    graphed.step_ctr.zero_()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        graphed.step(rt, yn)
    for _ in range(5):
        eager.step(rt, yn)
        g.replay()
    torch.cuda.synchronize()
    assert int(graphed.step_ctr.item()) == 5
    torch.testing.assert_close(graphed.P, eager.P, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("H", [64, 128, 256])
@pytest.mark.parametrize("B", [1000, 65536])
def test_fused_reduce_adamw_bitwise_equals_two_kernels(H, B, monkeypatch):
    """reduce_adamw (the one-rank step tail) == wgrad_reduce + adamw_pack, bit for bit: the
    gradient bucket, the master weights, both moments and the training blob, over 4 steps."""
    m = _model(H, 5)
    rt, yn = _batch(B, m, 6)
    rt, yn = rt.to(DEV), yn.to(DEV)
    kw = dict(lr=2e-3, weight_decay=0.01, warmup=2, total_steps=10, allreduce=False)
    fused = FusedMlp3Trainer(copy.deepcopy(m), DEV, B, B, **kw)
    split = FusedMlp3Trainer(copy.deepcopy(m), DEV, B, B, **kw)
    assert fused._local_only()
    for _ in range(4):
        monkeypatch.setenv("ROUTEST_FUSED_ADAMW", "1")
        fused.step(rt, yn)
        monkeypatch.setenv("ROUTEST_FUSED_ADAMW", "0")
        split.step(rt, yn)
    torch.cuda.synchronize()
    for name in ("G", "P", "M", "V", "blob", "step_ctr"):
        a, b = getattr(fused, name), getattr(split, name)
        assert torch.equal(a, b), name
    assert not torch.equal(fused.P.cpu(), flatten_params(m))


@pytest.mark.parametrize("K,M,Mout,N,S", [(65536, 256, 256, 272, 256), (1000, 256, 256, 272, 7),
                                           (4133, 8, 1, 272, 16), (777, 256, 200, 16, 3),
                                           (64, 64, 64, 96, 1)])
def test_wgrad_kernel_vs_fp32(K, M, Mout, N, S):
    from routest_amd.ops import _ext
    C = _ext.native()
    g = torch.Generator().manual_seed(K)
    A = torch.randn(K, M, generator=g).to(torch.bfloat16)
    Bm = torch.randn(K, N + 8, generator=g).to(torch.bfloat16)   # ldb > N
    ref = (A.float().t() @ Bm.float()[:, :N])[:Mout]
    ldo = N + 4
    stride = Mout * ldo + 16
    slab = torch.full((S, stride), float("nan"), device=DEV)
    C.wgrad(A.to(DEV), M, Mout, Bm.to(DEV), N, slab, 8, ldo)
    G = torch.zeros(stride, device=DEV)
    C.wgrad_reduce(slab[:, :], G)
    got = G[8:8 + Mout * ldo].view(Mout, ldo)[:, :N].cpu()
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-3 * (K ** 0.5))


@pytest.mark.parametrize("K,H,S", [(8192, 1024, 16), (4096, 512, 8), (65536, 1024, 16), (2048, 256, 3)])
def test_wgrad256_vs_fp32(K, H, S):
    """The wide trainer's dW2|db2 on 256 x 256 output tiles (wgrad.hip wgrad256_kernel): fragments
    through ds_read_b64_tr_b16 from swizzled stage images, split-K into slabs, db2 as per-tile-column
    partial column sums folded by wgrad_reduce — against fp32 A^T B and A.sum(0)."""
    from routest_amd.ops import _ext
    C = _ext.native()
    g = torch.Generator().manual_seed(K + H)
    ldg = H + 16
    A = torch.randn(K, H, generator=g).to(torch.bfloat16)
    Bm = torch.randn(K, ldg, generator=g).to(torch.bfloat16)
    Bm[:, H] = 1.0
    Bm[:, H + 1:] = 0.0
    ref = A.float().t() @ Bm.float()[:, :H]
    slab = torch.zeros(S, H * ldg, device=DEV)
    C.wgrad256(A.to(DEV), Bm.to(DEV), H, H, slab, ldg, H)
    G = torch.full((H * ldg,), float("nan"), device=DEV)
    C.wgrad_reduce(slab, G, fold_ld=ldg, fold_col=H)
    G2 = torch.full((H * ldg,), float("nan"), device=DEV)
    C.wgrad_reduce(slab, G2, fold_ld=ldg, fold_col=H)
    got = G.view(H, ldg).cpu()
    torch.testing.assert_close(got[:, :H], ref, rtol=1e-4, atol=1e-3 * (K ** 0.5))
    torch.testing.assert_close(got[:, H], A.float().sum(0), rtol=1e-4, atol=1e-3 * (K ** 0.5))
    assert torch.equal(got[:, H + 1:], torch.zeros(H, 15))
    assert torch.equal(G, G2)                        # deterministic (fixed-order reduce)


@pytest.mark.parametrize("S,n,stride", [(256, 74000, 74000), (37, 1001, 1003), (5, 4096, 4100), (1, 3, 3)])
def test_wgrad_reduce_exact_and_deterministic(S, n, stride):
    from routest_amd.ops import _ext
    C = _ext.native()
    g = torch.Generator().manual_seed(S * 7 + n)
    slab = torch.randn(S, stride, generator=g)
    G1 = torch.zeros(n, device=DEV)
    G2 = torch.zeros(n, device=DEV)
    sd = slab.to(DEV)
    C.wgrad_reduce(sd, G1)      # slab rows may be longer than the bucket
    C.wgrad_reduce(sd, G2)
    ref = slab.double().sum(0)[:n].float()
    torch.testing.assert_close(G1.cpu(), ref, rtol=1e-5, atol=1e-4)
    assert torch.equal(G1, G2)


def test_fused_training_bitwise_deterministic():
    """Two trainers from the same init on the same batches end bit-identical (fixed-order slab
    reduction, no atomics in the gradient path) — SURVEY §5.2 determinism check."""
    from routest_amd.data.synth import synth_records, synth_trips
    from routest_amd.models.mlp3 import EtaMLP
    from routest_amd.ops.eta_mlp import records_to_tensor
    from routest_amd.train.fused import FusedMlp3Trainer
    xs, ys = synth_trips(20000, 0)
    rec, y = synth_records(16384, 5)
    rt = records_to_tensor(rec).to(DEV)
    Ps = []
    for _ in range(2):
        torch.manual_seed(0)
        m = EtaMLP(256)
        m.fit_normalization(xs, ys)
        tr = FusedMlp3Trainer(m, DEV, 16384, 16384, lr=1e-3, allreduce=False)
        yn = tr.normalize_targets(torch.from_numpy(y).to(DEV))
        for _ in range(4):
            tr.step(rt, yn)
        torch.cuda.synchronize()
        Ps.append(tr.P.clone())
    assert torch.equal(Ps[0], Ps[1])


@pytest.mark.parametrize("K,S", [(65536, 256), (1000, 7), (40, 1)])
def test_wgrad_masked_relu_backward(K, S):
    """dW1 path: wgrad(dh1, x, mask=h1a) == ((dh1 * (h1 > 0))^T x) in fp32."""
    from routest_amd.ops import _ext
    C = _ext.native()
    g = torch.Generator().manual_seed(K)
    H = 256
    dh1 = torch.randn(K, H, generator=g).to(torch.bfloat16)
    h1a = torch.randn(K, H + 16, generator=g).to(torch.bfloat16)
    h1a[:, :H][torch.rand(K, H, generator=g) < 0.1] = 0.0          # exact zeros are masked too
    x = torch.randn(K, 16, generator=g).to(torch.bfloat16)
    ref = ((dh1.float() * (h1a[:, :H].float() > 0)).t() @ x.float())
    slab = torch.zeros(S, H * 16, device=DEV)
    C.wgrad(dh1.to(DEV), H, H, x.to(DEV), 16, slab, 0, 16, h1a.to(DEV))
    G = torch.zeros(H * 16, device=DEV)
    C.wgrad_reduce(slab, G)
    torch.testing.assert_close(G.view(H, 16).cpu(), ref, rtol=1e-4, atol=1e-3 * (K ** 0.5))


@pytest.mark.parametrize("K,S", [(65536, 256), (1000, 7)])
def test_wgrad_masked_hperm_columns(K, S):
    """Trainer's dW1 path: A (dh1) in natural unit order, mask (h1a) in the hperm order."""
    from routest_amd.ops import _ext
    from routest_amd.train.fused import hperm
    C = _ext.native()
    g = torch.Generator().manual_seed(K + 1)
    H = 256
    dh1 = torch.randn(K, H, generator=g).to(torch.bfloat16)
    h1 = torch.randn(K, H, generator=g).clamp_min(0).to(torch.bfloat16)      # natural order
    h1a = torch.zeros(K, H + 16, dtype=torch.bfloat16)
    h1a[:, :H] = h1[:, hperm(H)]                                             # stored order
    x = torch.randn(K, 16, generator=g).to(torch.bfloat16)
    ref = ((dh1.float() * (h1.float() > 0)).t() @ x.float())
    slab = torch.zeros(S, H * 16, device=DEV)
    C.wgrad(dh1.to(DEV), H, H, x.to(DEV), 16, slab, 0, 16, h1a.to(DEV), mask_hperm=True)
    G = torch.zeros(H * 16, device=DEV)
    C.wgrad_reduce(slab, G)
    torch.testing.assert_close(G.view(H, 16).cpu(), ref, rtol=1e-4, atol=1e-3 * (K ** 0.5))


@pytest.mark.parametrize("H", [512, 1024])
@pytest.mark.parametrize("B", [1000, 4096])
def test_wide_trainer_gradients_match_autograd(H, B):
    """H = 512 / 1024: the L2-streamed training step (csrc/mlp_big.hip) vs fp32 autograd."""
    from routest_amd.train.fused import FusedMlp3TrainerBig
    m = _model(H)
    rt, yn = _batch(B, m)
    tr = FusedMlp3Trainer(m, DEV, B, B)
    assert isinstance(tr, FusedMlp3TrainerBig)
    tr.forward_backward(rt.to(DEV), yn.to(DEV))
    torch.cuda.synchronize()
    got = grads_from_bucket(tr.G, H)
    ref_m = copy.deepcopy(m)
    loss = torch.nn.functional.mse_loss(ref_m.forward_normalized(featurize_torch(rt)), yn)
    loss.backward()
    for name, p in ref_m.named_parameters():
        g, r = got[name].reshape(-1), p.grad.reshape(-1)
        rel = (g - r).norm() / r.norm().clamp_min(1e-12)
        assert rel < 3e-2, (name, float(rel))
    mse = float(tr.sq_err.sum()) / B
    assert abs(mse - float(loss)) / float(loss) < 2e-2


@pytest.mark.parametrize("H", [512, 1024])
@pytest.mark.parametrize("B", [1000, 65536])
def test_dgrad_dw1_epilogue_matches_stored_dh1(H, B, monkeypatch):
    """dW1 from the dgrad GEMM's epilogue (dh1 never stored) == the stored-dh1 + masked wgrad path:
    the same bf16 dz1 values, summed in another order (fp32); every other gradient bit-identical."""
    from routest_amd.train.fused import FusedMlp3TrainerBig
    m = _model(H, 7)
    rt, yn = _batch(B, m, 8)
    rt, yn = rt.to(DEV), yn.to(DEV)
    monkeypatch.setenv("ROUTEST_DW1_EPILOGUE", "1")
    epi = FusedMlp3Trainer(copy.deepcopy(m), DEV, B, B)
    monkeypatch.setenv("ROUTEST_DW1_EPILOGUE", "0")
    ref = FusedMlp3Trainer(copy.deepcopy(m), DEV, B, B)
    assert isinstance(epi, FusedMlp3TrainerBig) and epi.dw1_epi and not ref.dw1_epi
    epi.forward_backward(rt, yn)
    ref.forward_backward(rt, yn)
    torch.cuda.synchronize()
    ldg = H + 16
    w1 = H * ldg + ldg
    assert torch.equal(epi.G[:w1], ref.G[:w1])
    a, b = epi.G[w1:].view(H, 16).cpu(), ref.G[w1:].view(H, 16).cpu()
    torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5 * float(b.abs().max()))
    assert float(b.abs().max()) > 0


def test_wide_trainer_h1024_steps_and_serves():
    """A trainer step at H = 1024 runs end to end (optimizer included), the loss falls, and the
    trained weights serve through the wide inference path."""
    from routest_amd.ops.eta_mlp import EtaMlpKernel
    H, B = 1024, 8192
    m = _model(H, 3)
    rec, y = synth_records(B * 4, 12)
    rt = records_to_tensor(rec).to(DEV)
    yn = ((torch.from_numpy(y) - m.y_mean) / m.y_std).float().to(DEV)
    tr = FusedMlp3Trainer(m, DEV, B, B, lr=1e-3, warmup=5, total_steps=60)
    first = None
    for s in range(60):
        k = s % 4
        tr.step(rt[k * B:(k + 1) * B], yn[k * B:(k + 1) * B])
        if s == 0:
            first = tr.local_mse()
    last = tr.local_mse()
    assert last < 0.5 * first, (first, last)
    assert torch.isfinite(tr.P).all()
    model = tr.to_model()
    erec, ey = synth_records(4096, 13)
    pred = EtaMlpKernel(model, DEV)(records_to_tensor(erec).to(DEV)).cpu()
    with torch.no_grad():
        ref = model(torch.from_numpy(records_to_features(erec))).reshape(-1)
    torch.testing.assert_close(pred, ref, rtol=3e-2, atol=0.3)


@pytest.mark.parametrize("B", [8192, 65536])
def test_column_split_backward_matches_full_width(B):
    """train_bwd_kernel's column split (NBW = 1: workgroup pairs own half the h1 units each and
    write one slab per pair; chosen for H = 256 when the slab count is a multiple of 8) gives the
    gradients of the full-width kernel (NBW = 2, forced here with a slab count that is not a multiple
    of 8) up to fp32 summation order."""
    H = 256
    m = _model(H)
    rt, yn = _batch(B, m)
    tr = FusedMlp3Trainer(m, DEV, B, B)
    assert tr.S % 8 == 0, tr.S                        # the trainer runs the split
    tr.forward_backward(rt.to(DEV), yn.to(DEV))
    torch.cuda.synchronize()
    g_split = tr.G.clone()
    ldg = H + 16
    S = tr.S - 1                                      # not a multiple of 8: full-width launch
    slab2 = torch.empty(S, H * ldg, dtype=torch.float32, device=DEV)
    slab = torch.empty(S, H * 16, dtype=torch.float32, device=DEV)
    C = tr.C
    C.train_bwd(tr.xf, B, tr.blob, H, tr.dz2r, slab2, slab)
    C.wgrad_reduce(slab2, tr.G[:H * ldg], slab, tr.G[H * ldg + ldg:], tr.w3slab, tr.G[H * ldg:H * ldg + ldg],
                   perm_h=H)
    torch.cuda.synchronize()
    rel = (g_split - tr.G).norm() / tr.G.norm()
    assert rel < 1e-5, float(rel)
    got, ref = grads_from_bucket(g_split, H), grads_from_bucket(tr.G, H)
    for name in ref:
        r = (got[name] - ref[name]).norm() / ref[name].norm().clamp_min(1e-12)
        assert r < 1e-4, (name, float(r))
