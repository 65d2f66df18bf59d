"""Convex 8x flow upsampling (reference `core/raft.py:72-83`) -- HIP kernel + pure-torch oracle."""
import torch
import torch.nn.functional as F

from . import _ext


def torch_convex_upsample(flow, mask):
    """Reference-semantics implementation (also the CPU path)."""
    n, _, h, w = flow.shape
    m = mask.view(n, 1, 9, 8, 8, h, w)
    m = torch.softmax(m, dim=2)
    up = F.unfold(8 * flow, [3, 3], padding=1).view(n, 2, 9, 1, 1, h, w)
    up = torch.sum(m * up, dim=2)
    up = up.permute(0, 1, 4, 2, 5, 3)
    return up.reshape(n, 2, 8 * h, 8 * w)


class _ConvexUpsample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flow, mask, nhwc):
        flow = flow.contiguous().float()
        mask = mask.contiguous()
        # fp16 masks (fp16 autocast) run on the NHWC kernels only
        if mask.dtype not in (torch.float32, torch.bfloat16) and not (nhwc and mask.dtype == torch.float16):
            mask = mask.float()
        ctx.save_for_backward(flow, mask)
        ctx.nhwc = nhwc
        return _ext.ops().convex_up_fwd(flow, mask, nhwc)

    @staticmethod
    def backward(ctx, dout):
        flow, mask = ctx.saved_tensors
        dflow, dmask = _ext.ops().convex_up_bwd(flow, mask, dout.contiguous().float(), ctx.nhwc)
        return dflow, dmask, None


def convex_upsample(flow, mask, impl='auto', nhwc=False):
    """``mask`` is (B,576,H,W), or (B,H,W,576) with ``nhwc=True`` (the fused update block's layout)."""
    if impl != 'torch' and _ext.device_ok(flow) and _ext.gpu_path_enabled(required=(impl == 'hip')):
        out_dtype = torch.promote_types(flow.dtype, mask.dtype)
        if (not nhwc and mask.dim() == 4 and not mask.is_contiguous() and
                mask.is_contiguous(memory_format=torch.channels_last)):
            # channels_last mask (the fp32 model's NHWC conv outputs): the NHWC kernel, no copy
            mask, nhwc = mask.permute(0, 2, 3, 1), True
        out = _ConvexUpsample.apply(flow, mask, nhwc)
        return out if out_dtype == torch.float32 else out.to(out_dtype)
    if nhwc:
        mask = mask.permute(0, 3, 1, 2)
    return torch_convex_upsample(flow, mask)
