"""Developer tool: per-parameter CNN gradient errors vs torch for several shapes."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_gpu_cnn as T  # noqa: E402
from oracle import ppo_ref as R  # noqa: E402
from surreal_amd import _lib as L  # noqa: E402
from tests.helpers import seq_flat  # noqa: E402

C, H, W = T.CAM
for (B, Tt, S, F) in [(24, 25, 26, 256), (624, 1, 1, 256), (24, 26, 26, 256), (12, 25, 26, 256),
                      (24, 25, 25, 256)]:
    torch.manual_seed(1)
    net = R.cnn_stem_ref(C, H, W, F)
    net64 = R.cnn_stem_ref(C, H, W, F).double()
    net64.load_state_dict({k: v.double() for k, v in net.state_dict().items()})
    flat = seq_flat(net).to('cuda')
    pix, pixn = T._images(B, Tt, S)
    rows = S * B
    x = T._timemajor_images(pix, pixn, S)
    pix_d, pixn_d = pix.cuda(), pixn.cuda()
    a1, a2, feat = T._run_fwd(flat, pix_d, pixn_d, B, Tt, rows, F)
    out = net(x / 255.0)
    dy = torch.randn(rows, F, generator=torch.Generator().manual_seed(7))
    dz = (dy * (out.detach() > 0)).cuda().contiguous()
    nbytes = int(L.lib().smi_cnn_scratch_bytes(rows, C, H, W, F))
    scratch = torch.empty(nbytes // 4 + 1, device='cuda')
    grad = torch.full_like(flat, float('nan'))
    L.call('smi_cnn_backward', L.ptr(flat), L.ptr(pix_d), L.ptr(pixn_d), B, Tt, rows,
           C, H, W, F, L.ptr(a1), L.ptr(a2), L.ptr(dz), F, L.ptr(grad), L.ptr(scratch), nbytes,
           L.stream())
    (out * dy).sum().backward()
    (net64(x.double() / 255.0) * dy.double()).sum().backward()
    got = grad.cpu()
    r1 = torch.relu(net[0](x / 255.0)).detach().reshape(rows, -1)
    a1e = float((a1.cpu().reshape(rows, -1) - r1).abs().max())
    p1 = torch.relu(net[0](x / 255.0)).detach()
    p2 = net[2](p1).detach().requires_grad_(True)
    o2 = torch.relu(net[5](net[4](torch.relu(p2))))
    (o2 * dy).sum().backward()
    dA2 = scratch[:rows * 2592].reshape(rows, 2592).cpu()
    d2e = (dA2 - p2.grad.reshape(rows, -1)).abs().amax(1)
    bad = torch.nonzero(d2e > 1e-4).flatten()
    print('  a1 err', a1e, 'dA2 err', float(d2e.max()), 'bad rows', bad[:10].tolist(), len(bad))
    o = 0
    errs = []
    for p, p64 in zip(net.parameters(), net64.parameters()):
        n = p.numel()
        sc = float(p64.grad.abs().max())
        e = float((got[o:o + n].reshape(p.shape).double() - p64.grad).abs().max() / sc)
        e32 = float((p.grad.double() - p64.grad).abs().max() / sc)
        errs.append((round(e, 8), round(e32, 8)))
        o += n
    print((B, Tt, S, F), 'feat err', float((feat.cpu() - out.detach()).abs().max()), 'grads', errs,
          flush=True)
