"""Training-step building blocks (csrc/train.hip) against torch fp32 autograd of the same
ops: train-mode Conv1x1 + BatchNorm + ReLU forward / backward, running statistics, the
weight-gradient GEMM, Adam.  Tolerances: forward 1e-4, gradients rtol 1e-3 (different
summation orders over up to 10^5 rows); the HIP reductions are also bitwise repeatable."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from pcd_reg_hregnet_amd import _lib as L
    L.load()
    yield


def _ref(x, W, bias, gamma, beta, rm, rv, relu):
    y = x @ W.t()
    if bias is not None:
        y = y + bias
    y = F.batch_norm(y, rm, rv, gamma, beta, training=True, momentum=0.1, eps=1e-5)
    return F.relu(y) if relu else y


@pytest.mark.parametrize("R,K,N,bias,relu", [(4096, 68, 64, False, True), (1000, 36, 20, True, True),
                                             (65536, 4, 32, False, True), (512, 256, 128, True, False)])
def test_conv_bn_act_matches_torch(R, K, N, bias, relu):
    from pcd_reg_hregnet_amd.train import conv_bn_act
    g = torch.Generator(device="cpu").manual_seed(R + K + N)
    x = (torch.randn(R, K, generator=g) * 2 + 0.5).cuda()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).cuda()
    b = torch.randn(N, generator=g).cuda() if bias else None
    gamma = (torch.rand(N, generator=g) + 0.5).cuda()
    beta = torch.randn(N, generator=g).cuda()
    G = torch.randn(R, N, generator=g).cuda()
    leaves = [t.clone().requires_grad_(True) for t in (x, W, gamma, beta)]
    bl = b.clone().requires_grad_(True) if bias else None
    rm, rv = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
    out = conv_bn_act(leaves[0], leaves[1], bl, leaves[2], leaves[3], rm, rv, relu)
    (out * G).sum().backward()
    tl = [t.clone().requires_grad_(True) for t in (x, W, gamma, beta)]
    tb = b.clone().requires_grad_(True) if bias else None
    trm, trv = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
    ref = _ref(tl[0], tl[1], tb, tl[2], tl[3], trm, trv, relu)
    (ref * G).sum().backward()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rm, trm, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv, trv, rtol=1e-5, atol=1e-6)
    for a, r, name in zip(leaves, tl, ("dx", "dW", "dgamma", "dbeta")):
        scale = float(r.grad.abs().max())
        torch.testing.assert_close(a.grad, r.grad, rtol=1e-3, atol=1e-4 * scale, msg=name)
    if bias:
        torch.testing.assert_close(bl.grad, tb.grad, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("bias", [False, True])
def test_conv_bn_act_accumulates_into_existing_grad_bitwise(bias):
    """A parameter used twice (src and dst pass) with its .grad pre-attached and zeroed
    (the trainer's gradient bucket): the backward adds dW / dbias / dgamma / dbeta into
    .grad itself (train._grad_slot) -- bitwise the gradients autograd's own accumulation
    gives when .grad starts as None."""
    from pcd_reg_hregnet_amd.train import conv_bn_act, direct_gradients
    g = torch.Generator(device="cpu").manual_seed(7)
    R, K, N = 8192, 36, 64
    xs = [(torch.randn(R, K, generator=g) * 2).cuda() for _ in range(2)]
    Gs = [torch.randn(R, N, generator=g).cuda() for _ in range(2)]
    W4 = (torch.randn(N, K, 1, 1, generator=g) / K ** 0.5).cuda()
    b = torch.randn(N, generator=g).cuda()
    gamma = (torch.rand(N, generator=g) + 0.5).cuda()
    beta = torch.randn(N, generator=g).cuda()
    grads = []
    for attach in (False, True):
        ps = [t.clone().requires_grad_(True) for t in (W4, b, gamma, beta)]
        if attach:
            for p in ps:
                p.grad = torch.zeros_like(p)
        loss = 0
        for x, G in zip(xs, Gs):
            rm, rv = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
            out = conv_bn_act(x, ps[0].view(N, K), ps[1] if bias else None, ps[2], ps[3], rm, rv,
                              True, wparam=ps[0])
            loss = loss + (out * G).sum()
        with direct_gradients():
            loss.backward()
        grads.append([p.grad.clone() if p.grad is not None else None for p in ps])
    for a, r, name in zip(grads[1], grads[0], ("dW", "dbias", "dgamma", "dbeta")):
        if name == "dbias" and not bias:
            assert r is None and not a.abs().max() > 0
            continue
        assert torch.equal(a, r), name


@pytest.mark.parametrize("R,K,N", [(40000, 32, 192), (40000, 4, 32), (33000, 36, 68), (20000, 192, 32),
                                   (17000, 384, 64), (16384, 128, 256), (16400, 68, 64)])
@pytest.mark.parametrize("w_trans", [False, True])
def test_ts_gemm_bitwise_equals_gemm(R, K, N, w_trans):
    """hreg_ts_gemm (tall-skinny training conv GEMM) gives hreg_gemm's bits: the same k-order,
    with W [N][K] or the transposed layout [K][N] read in place; ragged R, K % 16 != 0, N % 32
    != 0, bias shift, several column groups (K = 384)."""
    from pcd_reg_hregnet_amd import _lib, train
    g = torch.Generator(device="cpu").manual_seed(R + K + N)
    x = torch.randn(R, K, generator=g).cuda()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).cuda()
    b = torch.randn(N, generator=g).cuda()
    assert _lib.load().hreg_ts_gemm_supported(R, K, N, 0)
    ref = train._plain_gemm(x, W, b)
    Wl = W.t().contiguous() if w_trans else W  # [K][N]: the dx GEMM's layout
    out = torch.empty(R, N, device="cuda")
    _lib.call("hreg_ts_gemm", x, K, R, K, Wl, 1 if w_trans else 0, N, None, b, 0, out, N,
              _lib.stream_handle())
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert torch.equal(train._conv_gemm(x, Wl, b, w_trans=w_trans), ref)


@pytest.mark.parametrize("R,K,N", [(40000, 32, 192), (40000, 4, 32), (33000, 36, 68), (17000, 384, 64),
                                   (16384, 128, 256)])
def test_ts_gemm_bn_statistics(R, K, N):
    """hreg_ts_gemm_bn: y bitwise hreg_ts_gemm's; mean / invstd / unbiased var and the running
    update as hreg_bn_stats + hreg_bn_running_update (fp64 sums in another fixed order: equal
    to within an fp32 ulp); bitwise repeatable."""
    from pcd_reg_hregnet_amd import _lib, train
    g = torch.Generator(device="cpu").manual_seed(R + K)
    x = (torch.randn(R, K, generator=g) * 3 + 1).cuda()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).cuda()
    b = torch.randn(N, generator=g).cuda()
    rm0, rv0 = torch.randn(N, generator=g).cuda(), (torch.rand(N, generator=g) + 0.5).cuda()
    y_ref = train._conv_gemm(x, W, b)
    m_ref, i_ref, v_ref = train.bn_stats(y_ref, 1e-5)
    rm_ref, rv_ref = rm0.clone(), rv0.clone()
    _lib.call("hreg_bn_running_update", m_ref, v_ref, N, 0.1, rm_ref, rv_ref, _lib.stream_handle())
    outs = []
    for _ in range(2):
        rm, rv = rm0.clone(), rv0.clone()
        y, m, i, v = train._conv_gemm_bn(x, W, b, 1e-5, 0.1, rm, rv)
        outs.append((y, m, i, v, rm, rv))
    torch.cuda.synchronize()
    y, m, i, v, rm, rv = outs[0]
    assert torch.equal(y, y_ref)
    for a, r in ((m, m_ref), (i, i_ref), (v, v_ref), (rm, rm_ref), (rv, rv_ref)):
        torch.testing.assert_close(a, r, rtol=2e-7, atol=1e-7)
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)


def test_gemm_tn_and_transpose():
    from pcd_reg_hregnet_amd.train import gemm_tn, transpose
    g = torch.Generator(device="cpu").manual_seed(3)
    for R, N, K in ((1000, 70, 36), (70000, 64, 4), (33, 1, 5), (4096, 256, 260)):
        A = torch.randn(R, N, generator=g).cuda()
        B = torch.randn(R, K, generator=g).cuda()
        out = gemm_tn(A, B)
        ref = A.double().t() @ B.double()
        torch.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-3 * R ** 0.5 / 100)
        assert torch.equal(gemm_tn(A, B), out)  # deterministic
        assert torch.equal(transpose(A), A.t().contiguous())


@pytest.mark.parametrize("R,N,K", [(70000, 64, 64), (4096, 64, 32), (1000, 32, 32), (12345, 128, 260), (64, 96, 8)])
def test_gemm_tn_lds_staged_bitwise(R, N, K):
    """r6: the 16-byte-row LDS-staged weight-gradient kernel (gemm_tn4_kernel, taken when row
    strides and bases are 16-byte aligned) gives the dword-load kernel's bits (taken here through
    row strides N + 1, K + 1: the same rows in the same k-step order per wave)."""
    from pcd_reg_hregnet_amd.train import gemm_tn
    g = torch.Generator(device="cpu").manual_seed(R + N + K)
    A = torch.randn(R, N, generator=g).cuda()
    B = torch.randn(R, K, generator=g).cuda()
    A1 = torch.zeros(R, N + 1, device="cuda")[:, :N]
    B1 = torch.zeros(R, K + 1, device="cuda")[:, :K]
    A1.copy_(A)
    B1.copy_(B)
    assert A1.stride(0) % 4 and B1.stride(0) % 4
    staged, plain = gemm_tn(A, B), gemm_tn(A1, B1)
    assert torch.equal(staged, plain)
    ref = A.double().t() @ B.double()
    torch.testing.assert_close(staged.double(), ref, rtol=1e-4, atol=1e-3 * R ** 0.5 / 100)


def test_bn_stats_deterministic_and_accurate():
    from pcd_reg_hregnet_amd.train import bn_stats
    y = (torch.randn(300000, 48, generator=torch.Generator().manual_seed(1)) * 3 + 100).cuda()
    m, inv, var = bn_stats(y)
    m2, inv2, var2 = bn_stats(y)
    assert torch.equal(m, m2) and torch.equal(inv, inv2) and torch.equal(var, var2)
    yd = y.double()
    torch.testing.assert_close(m.double(), yd.mean(0), rtol=1e-7, atol=1e-6)
    torch.testing.assert_close(var.double(), yd.var(0, unbiased=True), rtol=1e-5, atol=0)
    torch.testing.assert_close(inv.double(), 1 / torch.sqrt(yd.var(0, unbiased=False) + 1e-5),
                               rtol=1e-5, atol=0)


def test_adam_matches_torch():
    from pcd_reg_hregnet_amd.train import Adam
    g = torch.Generator().manual_seed(7)
    p0 = [torch.randn(33, 17, generator=g).cuda(), torch.randn(1000, generator=g).cuda()]
    ours = [torch.nn.Parameter(p.clone()) for p in p0]
    ref = [torch.nn.Parameter(p.clone()) for p in p0]
    opt = Adam(ours, lr=1e-3)
    topt = torch.optim.Adam(ref, lr=1e-3)
    for step in range(5):
        grads = [torch.randn(p.shape, generator=g).cuda() * (step + 1) for p in p0]
        opt.zero_grad()
        topt.zero_grad()
        for p, q, gr in zip(ours, ref, grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        opt.step()
        topt.step()
    for p, q in zip(ours, ref):
        torch.testing.assert_close(p.data, q.data, rtol=1e-6, atol=1e-7)


def test_train_layer_stack_step():
    """Two ConvBNAct layers + Adam: three steps run, loss decreases, the HIP gradients of
    the stack match torch autograd of the same modules at step 1."""
    from pcd_reg_hregnet_amd.train import Adam, ConvBNAct
    torch.manual_seed(0)
    l1, l2 = ConvBNAct(36, 64).cuda(), ConvBNAct(64, 32, bias=True).cuda()
    x = torch.randn(2048, 36).cuda()
    target = torch.randn(2048, 32).cuda()
    params = list(l1.parameters()) + list(l2.parameters())
    opt = Adam(params, lr=1e-2)
    losses = []
    for _ in range(3):
        opt.zero_grad()
        out = l2(l1(x))
        loss = ((out - target) ** 2).mean()
        loss.backward()
        losses.append(float(loss))
        opt.step()
    assert losses[2] < losses[0]
    assert np.isfinite(losses).all()
