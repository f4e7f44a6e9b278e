"""The fused head passes (head_kernels.hip) through the C ABI against torch:
smi_head_forward (Linear-ReLU-Linear-ReLU-Linear[-Tanh], builders.py:86-175)
and smi_head_backward_input (the input-gradient chain of the same MLP, the
ReLU masks taken from the GPU's own forward activations: a pre-activation
within rounding distance of 0 may land either side in any two fp32
implementations, and the backward is linear given the masks).  Bar: within 2x
torch-CPU fp32's own error against fp64 and 1e-5 of the tensor's scale
(test_gpu_ddpg._fp32_as_good_as_torch), at the C3 widths (LSTM 100 -> 300 ->
200 -> 8 / 1) over the one-rank-of-eight (2688 rows) and full (21504 rows)
batches, and at ragged / narrow shapes."""
import pytest
import torch

from surreal_amd import _lib as L
from tests.test_gpu_ddpg import _fp32_as_good_as_torch

pytestmark = pytest.mark.gpu


def _flat(W1, b1, W2, b2, W3, b3):
    return torch.cat([W1.reshape(-1), b1, W2.reshape(-1), b2, W3.reshape(-1), b3]).float()


@pytest.mark.parametrize('rows,din,h1,h2,out,tanh_out', [
    (2688, 100, 300, 200, 8, 1), (21504, 100, 300, 200, 1, 0), (37, 20, 36, 28, 3, 0),
    (1, 16, 64, 48, 16, 1), (4099, 64, 32, 64, 6, 1), (513, 100, 300, 200, 8, 0)])
def test_head_forward_backward_vs_torch(rows, din, h1, h2, out, tanh_out):
    g = torch.Generator().manual_seed(rows + din + h1)
    lins = [torch.nn.Linear(din, h1), torch.nn.Linear(h1, h2), torch.nn.Linear(h2, out)]
    (W1, b1), (W2, b2), (W3, b3) = ((l.weight.detach(), l.bias.detach()) for l in lins)
    x = torch.randn(rows, din, generator=g)
    dz = torch.randn(rows, out, generator=g)
    P = _flat(W1, b1, W2, b2, W3, b3).cuda()
    xd, dzd = x.cuda(), dz.cuda()
    ha1 = torch.empty(rows, h1, device='cuda')
    ha2 = torch.empty(rows, h2, device='cuda')
    y = torch.empty(rows, out, device='cuda')
    wT = torch.empty(din * h1 + h1 * h2, device='cuda')
    st = L.stream()
    L.call('smi_head_forward', L.ptr(P), din, h1, h2, out, tanh_out, L.ptr(xd), din, rows,
           L.ptr(ha1), L.ptr(ha2), L.ptr(y), L.ptr(wT), st)
    torch.cuda.synchronize()
    # the transposes the backward reads
    assert torch.equal(wT[:din * h1].view(din, h1).cpu(), W1.t())
    assert torch.equal(wT[din * h1:].view(h1, h2).cpu(), W2.t())

    def fwd(dt):
        a1 = torch.relu(x.to(dt) @ W1.to(dt).t() + b1.to(dt))
        a2 = torch.relu(a1 @ W2.to(dt).t() + b2.to(dt))
        z = a2 @ W3.to(dt).t() + b3.to(dt)
        return a1, a2, torch.tanh(z) if tanh_out else z
    r32, r64 = fwd(torch.float32), fwd(torch.float64)
    for got, e32, e64 in zip((ha1, ha2, y), r32, r64):
        _fp32_as_good_as_torch(got.cpu(), e32, e64)
    # backward from dz with the GPU's masks, dX over columns [2, 2 + dxn)
    m1, m2 = (ha1 > 0).cpu(), (ha2 > 0).cpu()
    dx0 = 2 if din > 8 else 0
    dxn = din - dx0
    dh2 = torch.empty(rows, h2, device='cuda')
    dh1 = torch.empty(rows, h1, device='cuda')
    dx = torch.full((rows, dxn), float('nan'), device='cuda')
    L.call('smi_head_backward_input', L.ptr(P), din, h1, h2, out, L.ptr(wT), L.ptr(dzd), rows,
           L.ptr(ha1), L.ptr(ha2), L.ptr(dh2), L.ptr(dh1), dx0, dxn, L.ptr(dx), dxn, None, 0, st)

    def bwd(dt):
        d2 = (dz.to(dt) @ W3.to(dt)) * m2
        d1 = (d2 @ W2.to(dt)) * m1
        return d2, d1, d1 @ W1.to(dt)[:, dx0:dx0 + dxn]
    b32, b64 = bwd(torch.float32), bwd(torch.float64)
    for got, e32, e64 in zip((dh2, dh1, dx), b32, b64):
        _fp32_as_good_as_torch(got.cpu(), e32, e64)
    # with a mask on dX (the MLP policy's CNN-feature columns)
    mask = torch.randn(rows, dxn, generator=g).cuda()
    L.call('smi_head_backward_input', L.ptr(P), din, h1, h2, out, L.ptr(wT), L.ptr(dzd), rows,
           L.ptr(ha1), L.ptr(ha2), L.ptr(dh2), L.ptr(dh1), dx0, dxn, L.ptr(dx), dxn, L.ptr(mask),
           dxn, st)
    mk = (mask > 0).cpu()
    _fp32_as_good_as_torch(dx.cpu(), b32[2] * mk, b64[2] * mk)


def test_head_rejects_unsupported_shapes():
    P = torch.zeros(10000, device='cuda')
    x = torch.zeros(8, 17, device='cuda')
    o = torch.empty(8, 64, device='cuda')
    rc = L.lib().smi_head_forward(L.ptr(P), 17, 32, 32, 2, 0, L.ptr(x), 17, 8, L.ptr(o), L.ptr(o),
                                  L.ptr(o), None, L.stream())
    assert rc == -2            # SMI_E_NOFIT: in % 4 != 0
