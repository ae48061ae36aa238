"""Debug: bf16 GatedResBlock (fused node / per-op native / pure torch fp32) - where do they differ?"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from applestar_amd import ops
    from applestar_amd.ops import native as N
    from applestar_amd.models.blocks import GatedResBlock
    N.ensure_loaded()
    N.GATE_CHAIN = False
    torch.manual_seed(19)
    C = 128
    blk = GatedResBlock(C).cuda().to(memory_format=torch.channels_last)
    with torch.no_grad():
        blk.UpdateSP.fill_(0.7)
    x = torch.randn(4, C, 19, 20, device='cuda').to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        out = blk(x)
        y = blk.conv2(blk.conv1(x))
        g = blk.GateWeightG(x)
        ref = ops.gated_residual(y, g, blk.UpdateSP, x)
    # pure torch fp32 on bf16-rounded weights
    xf = x.float()
    w = lambda m: m[0].weight.to(torch.bfloat16).float()
    b = lambda m: m[0].bias.float()
    yt = F.conv2d(F.relu(F.conv2d(xf, w(blk.conv1), b(blk.conv1), padding=1)), w(blk.conv2), b(blk.conv2), padding=1)
    h = xf
    for i, m in enumerate(blk.GateWeightG):
        h = F.conv2d(h, w(m), b(m))
        if i < 3:
            h = F.relu(h)
    gt = h
    rt = torch.relu(torch.tanh(yt * torch.sigmoid(gt)) * 0.7 + xf)

    def d(a, bb, name):
        e = (a.float() - bb.float()).abs()
        idx = torch.nonzero(e == e.max())[0].tolist()
        print(f'{name}: max {e.max().item():.4f} at {idx} ({a.float()[tuple(idx)].item():.4f} vs '
              f'{bb.float()[tuple(idx)].item():.4f}), mean {e.mean().item():.5f}', flush=True)
    d(y, yt, 'per-op conv path vs torch')
    d(g, gt, 'per-op gate path vs torch')
    d(ref, rt, 'per-op block vs torch')
    d(out, rt, 'fused block vs torch')
    d(out, ref, 'fused vs per-op')


if __name__ == '__main__':
    main()
