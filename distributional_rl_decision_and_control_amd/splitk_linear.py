"""Linear layers whose weight gradient is reduced with a split-K batched GEMM.

In the IQN critic the rows are (sample, tau) pairs -- B*N = 131072 at the bench size -- so
each weight gradient dW = dY^T X is a GEMM with a tiny output (<= 256 x 256) and a huge
reduction dimension. A single GEMM call leaves most of the 256 CUs idle (rocprof showed
4-tile hipBLASLt kernels taking 200-320 us). Splitting the rows into G groups turns it into
one batched GEMM with G x more tiles plus a G-way sum, which fills the chip.
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

SPLITK_MIN_ROWS = 8192
SPLITK_GROUP_ROWS = int(os.environ.get("ASVRL_SPLITK_GROUP_ROWS", "512"))


def _groups(rows, group_rows=SPLITK_GROUP_ROWS):
    g = max(1, rows // group_rows)
    while rows % g:
        g -= 1
    return g


def _splitk_grads(ctx, x, weight, gy):
    gr = ctx.group_rows
    gx = gw = gb = None
    if ctx.needs_input_grad[0]:
        gx = gy.matmul(weight.to(gy.dtype))
    rows = x.shape[0]
    if ctx.needs_input_grad[1]:
        g = _groups(rows, gr)
        xs = x.reshape(g, rows // g, x.shape[1])
        ys = gy.reshape(g, rows // g, gy.shape[1])
        gw = torch.bmm(ys.transpose(1, 2), xs.to(ys.dtype)).sum(0, dtype=torch.float32).to(weight.dtype)
    if ctx.has_bias and ctx.needs_input_grad[2]:
        if _BIAS_TWO_STAGE:
            g = _groups(rows, gr)
            gb = gy.reshape(g, rows // g, gy.shape[1]).sum(1, dtype=torch.float32).sum(0).to(gy.dtype)
        else:
            gb = gy.sum(0, dtype=torch.float32).to(gy.dtype)
    return gx, gw, gb


class _SplitKLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, group_rows):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.group_rows = group_rows
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        return _splitk_grads(ctx, x, weight, gy) + (None,)


class _SplitKLinearReLU(torch.autograd.Function):
    """relu(F.linear(x, weight, bias)) with the bias + ReLU in the GEMM epilogue
    (torch._addmm_activation has no autograd formula of its own); fp32/bf16 2-D x, bias required."""

    @staticmethod
    def forward(ctx, x, weight, bias, group_rows):
        y = torch._addmm_activation(bias, x, weight.t())
        ctx.save_for_backward(x, weight, y)
        ctx.has_bias = True
        ctx.group_rows = group_rows
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, y = ctx.saved_tensors
        return _splitk_grads(ctx, x, weight, torch.ops.aten.threshold_backward(gy, y, 0)) + (None,)


ENABLED = os.environ.get("ASVRL_SPLITK", "1") != "0"
_BIAS_TWO_STAGE = os.environ.get("ASVRL_SPLITK_BIAS2", "1") == "1"  # rows -> groups -> 1 (rocprof: 2.09 -> 2.04 ms Rainbow step)


class SplitKLinear(nn.Linear):
    """nn.Linear (same parameters / state_dict) with the split-K weight gradient for large,
    2-D inputs; falls back to F.linear otherwise."""

    def forward(self, x):
        if ENABLED and x.dim() == 2 and x.shape[0] >= SPLITK_MIN_ROWS and torch.is_grad_enabled() and self.weight.requires_grad:
            if torch.is_autocast_enabled():
                dt = torch.get_autocast_gpu_dtype()
                with torch.autocast("cuda", enabled=False):
                    return _SplitKLinear.apply(x.to(dt), self.weight.to(dt), self.bias.to(dt), SPLITK_GROUP_ROWS)
            return _SplitKLinear.apply(x, self.weight, self.bias, SPLITK_GROUP_ROWS)
        return F.linear(x, self.weight, self.bias)


RowLinear = SplitKLinear  # the layers applied per (sample, tau) row
