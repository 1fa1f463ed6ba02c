"""DeepSpeech2 recurrent layers and CTC loss (ops/rnn.py; csrc/rnn.hip,
csrc/ctc.hip).

CPU tests pin the plain-PyTorch oracle: the LSTM recurrence (TF
BasicLSTMCell, gates i, j, f, o, forget bias 1.0) against torch.nn.LSTM with
re-ordered weights.  GPU tests run the HIP kernels against that fp32 oracle
(forward and every gradient) and the CTC kernel against torch's CTC loss.
"""

import pytest
import torch

from kf_benchmarks_amd.ops import rnn as R


def _to_torch_lstm(wx, bx, wh, H, d):
    """Our [din, 4H] / [H, 4H] (gates i, j, f, o) -> nn.LSTM's [4H, din]
    (gates i, f, g, o) for direction d, forget bias folded in."""
    G = 4 * H
    wxd, bxd, whd = wx[:, d * G:(d + 1) * G], bx[d * G:(d + 1) * G], wh[d]

    def reorder(m):
        i, j, f, o = m.split(H, dim=-1)
        return torch.cat([i, f, j, o], dim=-1)

    b = bxd.clone()
    b[2 * H:3 * H] += 1.0
    return reorder(wxd).t(), reorder(whd).t(), reorder(b)


@pytest.mark.parametrize("dirs", [1, 2])
def test_lstm_reference_matches_torch_lstm(dirs):
    torch.manual_seed(0)
    T, B, din, H = 6, 3, 5, 4
    x = torch.randn(T, B, din)
    wx = torch.randn(din, dirs * 4 * H) * 0.4
    bx = torch.randn(dirs * 4 * H) * 0.1
    wh = torch.randn(dirs, H, 4 * H) * 0.4
    gx = x.reshape(T * B, din) @ wx + bx
    ours = R.recurrence_reference(gx.view(T, B, -1), wh, R.LSTM, dirs, H)
    lstm = torch.nn.LSTM(din, H, bidirectional=dirs == 2)
    with torch.no_grad():
        for d in range(dirs):
            sfx = "_reverse" if d else ""
            wi, whh, b = _to_torch_lstm(wx, bx, wh, H, d)
            getattr(lstm, "weight_ih_l0" + sfx).copy_(wi)
            getattr(lstm, "weight_hh_l0" + sfx).copy_(whh)
            getattr(lstm, "bias_ih_l0" + sfx).copy_(b)
            getattr(lstm, "bias_hh_l0" + sfx).zero_()
        ref, _ = lstm(x)
    torch.testing.assert_close(ours, ref, rtol=1e-5, atol=1e-5)


def test_tanh_rnn_reference():
    torch.manual_seed(1)
    T, B, H = 5, 2, 3
    gx = torch.randn(T, B, H)
    wh = torch.randn(1, H, H) * 0.5
    out = R.recurrence_reference(gx, wh, R.TANH, 1, H)
    h = torch.zeros(B, H)
    for t in range(T):
        h = torch.tanh(gx[t] + h @ wh[0])
        torch.testing.assert_close(out[t], h)


def test_gru_reference_matches_tf_gru_cell_math():
    """TF GRUCell: r, u = sigmoid([x, h] Wg + bg); c = tanh([x, r h] Wc + bc);
    h' = u h + (1 - u) c, written out with the concatenated kernels."""
    torch.manual_seed(2)
    T, B, din, H = 4, 3, 5, 6
    x = torch.randn(T, B, din)
    kg = torch.randn(din + H, 2 * H) * 0.3
    kc = torch.randn(din + H, H) * 0.3
    bg, bc = torch.ones(2 * H), torch.zeros(H)
    wx = torch.cat([kg[:din], kc[:din]], 1)
    wh = torch.cat([kg[din:], kc[din:]], 1)[None]
    gx = x.reshape(T * B, din) @ wx + torch.cat([bg, bc])
    out = R.recurrence_reference(gx.view(T, B, -1), wh, R.GRU, 1, H)
    h = torch.zeros(B, H)
    for t in range(T):
        r, u = torch.sigmoid(torch.cat([x[t], h], 1) @ kg + bg).split(H, 1)
        c = torch.tanh(torch.cat([x[t], r * h], 1) @ kc + bc)
        h = u * h + (1 - u) * c
        torch.testing.assert_close(out[t], h, rtol=1e-5, atol=1e-5)


def test_permute01_cpu():
    x = torch.arange(24.).view(2, 3, 4)
    y = R.permute01(x)
    assert y.shape == (3, 2, 4) and torch.equal(y, x.transpose(0, 1))


# ------------------------------------------------------------------ GPU
def _relerr(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kind", [R.LSTM, R.TANH, R.GRU])
@pytest.mark.parametrize("dirs,B,H,T", [(2, 20, 32, 7), (1, 33, 48, 5), (2, 64, 160, 9)])
def test_recurrence_gpu(cuda, dt, kind, dirs, B, H, T):
    torch.manual_seed(0)
    G = R.GATES[kind]
    gx = torch.randn(T, B, dirs * G * H)
    wh = torch.randn(dirs, H, G * H) * (0.5 / H ** 0.5)
    dout = torch.randn(T, B, dirs * H)
    ga = gx.to(cuda, dt).requires_grad_(True)
    wa = wh.to(cuda).requires_grad_(True)
    out = R.recurrence(ga, wa, kind, dirs, H)
    out.backward(dout.to(cuda, dt))
    gb = gx.to(dt).float().requires_grad_(True)
    wb = wh.clone().requires_grad_(True)
    ref = R.recurrence_reference(gb, wb, kind, dirs, H)
    ref.backward(dout.to(dt).float())
    lim = 1e-4 if dt == torch.float32 else 3e-2
    assert _relerr(out, ref) < lim
    assert _relerr(ga.grad, gb.grad) < lim * 2
    assert _relerr(wa.grad, wb.grad) < lim * 2


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_rnn_layer_gpu(cuda, dt):
    """Input projection (affine GEMM) + recurrence, gradients of x, wx, bx, wh."""
    torch.manual_seed(3)
    T, B, din, H, dirs = 6, 16, 40, 32, 2
    x = torch.randn(T, B, din)
    wx = torch.randn(din, dirs * 4 * H) / din ** 0.5
    bx = torch.randn(dirs * 4 * H) * 0.1
    wh = torch.randn(dirs, H, 4 * H) / H ** 0.5
    dout = torch.randn(T, B, dirs * H)
    pa = [t.to(cuda).requires_grad_(True) for t in (wx, bx, wh)]
    xa = x.to(cuda, dt).requires_grad_(True)
    ya = R.rnn_layer(xa, pa[0], pa[1], pa[2], R.LSTM, dirs, H)
    ya.backward(dout.to(cuda, dt))
    pb = [t.clone().requires_grad_(True) for t in (wx, bx, wh)]
    xb = x.to(dt).float().requires_grad_(True)
    gx = xb.reshape(T * B, din) @ pb[0].to(dt).float() + pb[1]
    yb = R.recurrence_reference(gx.view(T, B, -1), pb[2], R.LSTM, dirs, H)
    yb.backward(dout.to(dt).float())
    lim = 1e-4 if dt == torch.float32 else 4e-2
    assert _relerr(ya, yb) < lim
    assert _relerr(xa.grad, xb.grad) < 2 * lim
    for a, b in zip(pa, pb):
        assert _relerr(a.grad, b.grad) < 2 * lim


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_ctc_gpu(cuda, dt):
    torch.manual_seed(0)
    B, T, C, L = 6, 40, 29, 12
    z = torch.randn(T, B, C) * 2  # time-major storage, [B, T, C] view as the model
    labels = torch.randint(0, C - 1, (B, L), dtype=torch.int32)
    labels[1, :4] = 5  # repeats need extra blanks
    ilen = torch.tensor([40, 31, 40, 25, 3, 40], dtype=torch.int32)   # seq 4 is infeasible
    llen = torch.tensor([12, 9, 1, 12, 12, 0], dtype=torch.int32)    # seq 5: empty label
    za = z.to(cuda, dt).requires_grad_(True)
    la = R.ctc_loss(za.transpose(0, 1), labels.to(cuda), ilen.to(cuda), llen.to(cuda))
    gl = torch.rand(B)
    la.backward(gl.to(cuda))
    zb = z.to(dt).float().requires_grad_(True)
    lb = R.ctc_loss_reference(zb.transpose(0, 1), labels, ilen, llen)
    lb.backward(gl)
    assert la[4].item() == 0.0 and lb[4].item() == 0.0
    torch.testing.assert_close(la.cpu(), lb.detach(), rtol=1e-4, atol=1e-4)
    # rows past each sequence end carry zero gradient on both sides
    torch.testing.assert_close(za.grad.float().cpu(), zb.grad, rtol=2e-2 if dt != torch.float32
                               else 1e-4, atol=1e-2 if dt != torch.float32 else 1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_ctc_loss_mean_gpu(cuda, dt):
    """The DeepSpeech2 loss as one native op: input lengths scaled on the
    device (ilen * T // max_time, the reference's arithmetic), CTC, batch
    mean and the mean's backward; vs torch's ctc_loss on the same scaled
    lengths (fp32 reference)."""
    torch.manual_seed(1)
    B, T, C, L, TMAX = 5, 48, 29, 10, 3494
    z = torch.randn(T, B, C) * 2
    labels = torch.randint(0, C - 1, (B, L), dtype=torch.int32)
    ilen = torch.tensor([[3494], [2000], [3494], [700], [80]], dtype=torch.int32)
    llen = torch.tensor([[10], [7], [1], [10], [5]], dtype=torch.int32)
    za = z.to(cuda, dt).requires_grad_(True)
    la = R.ctc_loss_mean(za.transpose(0, 1), labels.to(cuda), ilen.to(cuda), llen.to(cuda), T,
                         TMAX)
    la.backward(torch.tensor(1.5, device=cuda))
    zb = z.to(dt).float().requires_grad_(True)
    sl = (ilen.reshape(-1).long() * T) // TMAX
    lb = R.ctc_loss_reference(zb.transpose(0, 1), labels, sl, llen.reshape(-1)).mean()
    (lb * 1.5).backward()
    assert la.dim() == 0 and la.dtype == torch.float32
    torch.testing.assert_close(la.cpu(), lb.detach(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(za.grad.float().cpu(), zb.grad, rtol=2e-2 if dt != torch.float32
                               else 1e-4, atol=1e-2 if dt != torch.float32 else 1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_permute01_gpu(cuda, dt):
    x = torch.randn(7, 5, 3, 24)
    y = R.permute01(x.to(cuda, dt).requires_grad_(True))
    assert torch.equal(y.cpu(), x.to(dt).transpose(0, 1))


@pytest.mark.gpu
@pytest.mark.parametrize("rnn_type", ["lstm", "gru"])
def test_deepspeech2_small_gpu_matches_cpu(cuda, rnn_type):
    """Tiny DeepSpeech2 forward + backward on the GPU kernels (conv, BN,
    LSTM, affine, CTC) against the same model on CPU, fp32."""
    from kf_benchmarks_amd import datasets, params as P
    from kf_benchmarks_amd.models import model_config
    from kf_benchmarks_amd.models.model import make_network
    d = datasets.create_dataset(None, "librispeech")
    losses, grads = [], []
    cpu_inp = None
    for dev in ("cpu", cuda):
        m = model_config.get_model_config("deepspeech2", d, P.make_params(model="deepspeech2"))
        m.max_time_steps, m.max_label_length, m.rnn_hidden_size = 120, 20, 32
        m.rnn_type = rnn_type
        m.set_batch_size(4)
        torch.manual_seed(0)
        net = make_network(m, d.num_classes, str(dev), torch.float32)
        # the same inputs on both (the device draws its own synthetic stream)
        if cpu_inp is None:
            inp = cpu_inp = m.get_synthetic_inputs("x", d.num_classes, "cpu", 0)
        else:
            inp = tuple(t.to(dev) for t in cpu_inp)
        res = net.forward_inputs(inp)
        loss = m.loss_function(inp, res)
        loss.backward()
        losses.append(float(loss))
        grads.append(torch.cat([p.grad.reshape(-1).float().cpu() for p in net.parameters()
                                if p.grad is not None]))
    assert abs(losses[0] - losses[1]) < 1e-3 * abs(losses[0])
    assert _relerr(grads[1], grads[0]) < 1e-2
