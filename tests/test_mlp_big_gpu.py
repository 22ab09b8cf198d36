"""Wide MLPs (H = 512, 1024) on the L2-streamed path (csrc/mlp_big.hip) vs the PyTorch emulation
of its numerics and the fp32 model."""
import numpy as np
import pytest
import torch

from routest_amd.data.synth import synth_records
from routest_amd.models.features import records_to_features
from routest_amd.models.mlp3 import EtaMLP
from routest_amd.ops.eta_mlp import EtaMlpKernel, featurize_torch, records_to_tensor
from routest_amd.ops.mlp_big import emulate_big, hperm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _model(H, seed=0):
    torch.manual_seed(seed)
    m = EtaMLP(H)
    rec, y = synth_records(8192, seed)
    m.fit_normalization(records_to_features(rec), y)
    return m


@pytest.mark.parametrize("H", [512, 1024])
@pytest.mark.parametrize("B", [1, 127, 1000, 70_001])
def test_big_forward_matches_emulation_and_fp32(H, B):
    m = _model(H, 1)
    k = EtaMlpKernel(m, DEV)
    assert k._big is not None
    rec, _ = synth_records(B, 3)
    rt = records_to_tensor(rec)
    got = k(rt.to(DEV)).cpu()
    emu = emulate_big(k._big.packed, rt).reshape(-1)
    with torch.no_grad():
        ref = m(featurize_torch(rt)).reshape(-1)
    spread = max(float((ref - ref.mean()).abs().mean()), 1e-3) if B > 1 else 1.0
    assert torch.isfinite(got).all()
    assert float((got - emu).abs().max()) / spread < 5e-3          # accumulation order only
    torch.testing.assert_close(got, ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("H", [512, 1024])
def test_big_forward_trained_model(H):
    """Trained (fp32 autograd) wide model: error relative to the prediction spread."""
    torch.manual_seed(7)
    m = EtaMLP(H)
    rec, y = synth_records(1 << 15, 8)
    x = torch.from_numpy(records_to_features(rec))
    m.fit_normalization(x.numpy(), y)
    md = m.to(DEV)
    xd, yd = x.to(DEV), torch.from_numpy(y).to(DEV)
    yn = (yd - md.y_mean) / md.y_std
    opt = torch.optim.Adam(md.parameters(), lr=1e-3)
    for s in range(200):
        k0 = (s % 8) * 4096
        loss = torch.nn.functional.mse_loss(md.forward_normalized(xd[k0:k0 + 4096]), yn[k0:k0 + 4096])
        opt.zero_grad()
        loss.backward()
        opt.step()
    m = md.cpu().eval()
    erec, _ = synth_records(100_000, 9)
    got = EtaMlpKernel(m, DEV)(records_to_tensor(erec).to(DEV)).cpu()
    with torch.no_grad():
        ref = m(torch.from_numpy(records_to_features(erec))).reshape(-1)
    spread = (ref - ref.mean()).abs().mean()
    assert spread > 5.0
    err = (got - ref).abs() / spread
    assert float(err.max()) < 0.04 and float(err.mean()) < 0.006, (float(err.max()), float(err.mean()))


def test_big_forward_zero_copy_and_wire_formats():
    from routest_amd.models.features import records_to_compact6
    from routest_amd.ops.eta_mlp import records6_to_tensor
    m = _model(512, 2)
    k = EtaMlpKernel(m, DEV)
    rec, _ = synth_records(50_001, 4)
    rt = records_to_tensor(rec)
    ref = k(rt.to(DEV)).cpu()
    host = rt.pin_memory()
    out = torch.full((len(rec),), float("nan")).pin_memory()
    k.forward_hostio(host, out)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    r6 = records6_to_tensor(records_to_compact6(rec))
    got6 = k(r6.to(DEV)).cpu()
    assert (got6 - ref).abs().max() < 0.1                  # 6-byte record quantisation only


@pytest.mark.parametrize("M", [128, 1000, 4097])
def test_gemm_nt_store_epilogue(M):
    """EPI_STORE: out[m][hperm(n)] = sum_k W[n][k] X[m][k] (the dgrad GEMM of the wide trainer)."""
    from routest_amd.ops import _ext
    C = _ext.native()
    g = torch.Generator().manual_seed(M)
    N, K = 256, 512
    W = torch.randn(N, K, generator=g).to(torch.bfloat16)
    X = torch.randn(M, K, generator=g).to(torch.bfloat16)
    out = torch.zeros(M, N + 16, dtype=torch.bfloat16, device=DEV)
    C.gemm_nt(2, W.to(DEV), X.to(DEV), N, M, K, out=out)
    torch.cuda.synchronize()
    ref = (X.float() @ W.float().T)                    # [M, N] natural unit order
    got = torch.empty(M, N)
    got[:, hperm(N)] = out[:, :N].float().cpu()        # stored position c holds unit hperm(c)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=0.15)
    assert (out[:, N:] == 0).all()


@pytest.mark.parametrize("N,K,M", [(256, 64, 300), (256, 128, 256), (512, 192, 1000), (1024, 1024, 4097),
                                   (1024, 1024, 65536)])
def test_gemm_phase_pipeline_bitwise_equals_drain_loop(N, K, M):
    """gemm256p_kernel (phase pipeline, staggered wave groups, loads in flight across raw barriers)
    against gemm256_kernel (one drain per K-tile): the same MFMAs in the same per-accumulator order,
    so all three epilogues must agree bit for bit — including 1-, 2- and 3-K-tile loops (the
    prologue / tail waits) and a partial last row tile; and against torch."""
    from routest_amd.ops import _ext
    C = _ext.native()
    g = torch.Generator().manual_seed(N + K + M)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(DEV)
    X = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    b2 = (0.1 * torch.randn(N, generator=g)).to(DEV)
    w3 = (torch.randn(N, generator=g) / N ** 0.5).to(DEV)
    prev = C.gemm_pipe(-1)
    res = {}
    try:
        for pipe in (0, 1):
            C.gemm_pipe(pipe)
            o2 = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
            C.gemm_nt(2, W, X, N, M, K, out=o2)
            o1 = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
            y1 = torch.full((M, N // 64), float("nan"), device=DEV)
            C.gemm_nt(1, W, X, N, M, K, b2=b2, w3=w3, ypart=y1, out=o1)
            y0 = torch.full((M, N // 64), float("nan"), device=DEV)
            C.gemm_nt(0, W, X, N, M, K, b2=b2, w3=w3, ypart=y0)
            torch.cuda.synchronize()
            res[pipe] = (o2.cpu(), o1.cpu(), y1.cpu(), y0.cpu())
    finally:
        C.gemm_pipe(prev)
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a.view(torch.int32),
                           b.view(torch.int16) if b.dtype == torch.bfloat16 else b.view(torch.int32))
    z = (X.float() @ W.float().T).cpu()
    got = torch.empty(M, N)
    got[:, hperm(N)] = res[1][0].float()
    torch.testing.assert_close(got, z, rtol=1e-2, atol=0.05)
    y = (torch.relu(z + b2.cpu()) * w3.cpu()).view(M, N // 64, 64).sum(-1)
    torch.testing.assert_close(res[1][3], y, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("H", [512, 1024])
@pytest.mark.parametrize("rb", [16, 6])
def test_big_fused_equals_three_launch_path(H, rb):
    """The one-launch kernel (layer 1 computed in-register per K stage, h1 never in HBM) against
    the layer-1 kernel -> h1 -> GEMM path: same bf16 h1, same fp32 accumulation order per 32-k
    chunk up to the K permutation, so the two agree to accumulation-order rounding."""
    from routest_amd.models.features import records_to_compact6
    from routest_amd.ops.eta_mlp import records6_to_tensor
    from routest_amd.ops.mlp_big import EtaMlpBigKernel
    m = _model(H, 5)
    k = EtaMlpBigKernel(m, DEV)
    rec, _ = synth_records(33_333, 6)
    rt = records_to_tensor(rec) if rb == 16 else records6_to_tensor(records_to_compact6(rec))
    rd = rt.to(DEV)
    try:
        EtaMlpBigKernel.FUSED = False
        ref = k(rd).cpu()
        EtaMlpBigKernel.FUSED = True
        got = k(rd).cpu()
    finally:
        EtaMlpBigKernel.FUSED = True
    spread = float((ref - ref.mean()).abs().mean())
    assert torch.isfinite(got).all()
    assert float((got - ref).abs().max()) / spread < 2e-3
