"""Flat parameter storage: every nn.Parameter of a module becomes a view of one fp32 buffer, and
its .grad a view of one gradient buffer.  Clip-norm, the optimiser, the EMA and the data-parallel
gradient all-reduce then touch one contiguous allocation (one RCCL call per optimiser step), and
weights that are used as one concatenated operand (q|k|v|gate|mix, actor|critic heads) are laid out
adjacently so the concatenation — and its gradient — is a view, not a copy."""
from __future__ import annotations

import torch
from torch import nn


class FlatParams:
    def __init__(self, module: nn.Module, device, order=None, extra=0):
        """``extra`` floats follow the gradient buffer (``grad_ext = grad | extra``): per-step
        statistics stored there ride along in the same data-parallel all-reduce."""
        named = dict(module.named_parameters())
        order = list(order) if order is not None else list(named)
        assert sorted(order) == sorted(named), 'flat order must list every parameter exactly once'
        self.names = order
        self.params = [named[n] for n in order]
        sizes = [p.numel() for p in self.params]
        self.n = sum(sizes)
        self.flat = torch.empty(self.n, device=device, dtype=torch.float32)
        self.grad_ext = torch.zeros(self.n + extra, device=device, dtype=torch.float32)
        self.grad = self.grad_ext[:self.n]
        self.extra = self.grad_ext[self.n:]
        offs = [0]
        for s in sizes:
            offs.append(offs[-1] + s)
        self.offsets = offs
        self.index = {n: (a, b) for n, a, b in zip(order, offs[:-1], offs[1:])}
        for p, a, b in zip(self.params, offs[:-1], offs[1:]):
            self.flat[a:b].copy_(p.detach().reshape(-1).to(device))
            p.data = self.flat[a:b].view(p.shape)
            p.grad = self.grad[a:b].view(p.shape)
        self.seg = torch.tensor(offs, device=device, dtype=torch.int64)

    def zero_grad(self):
        self.grad.zero_()

    def span(self, names, buf=None):
        """Contiguous view covering ``names`` (which must be adjacent, in order) of flat or ``buf``."""
        buf = self.flat if buf is None else buf
        a0, b_prev = self.index[names[0]]
        for n in names[1:]:
            a, b = self.index[n]
            assert a == b_prev, f'{n} is not adjacent to its predecessor in the flat layout'
            b_prev = b
        return buf[a0:b_prev]

    def rebind(self, module: nn.Module, flat: torch.Tensor):
        """Point ``module``'s parameters (same names / shapes, e.g. an EMA copy) at ``flat``."""
        for n, p in module.named_parameters():
            a, b = self.index[n]
            p.data = flat[a:b].view(p.shape)
            p.requires_grad_(False)
