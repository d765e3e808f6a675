"""Flat parameter storage: every nn.Parameter of a module becomes a view of one fp32 buffer, and
its .grad a view of one gradient buffer.  Clip-norm, the optimiser, the EMA and the data-parallel
gradient all-reduce then touch one contiguous allocation (one RCCL call per optimiser step)."""
from __future__ import annotations

import torch
from torch import nn


class FlatParams:
    def __init__(self, module: nn.Module, device):
        self.params = [p for p in module.parameters()]
        self.names = [n for n, _ in module.named_parameters()]
        sizes = [p.numel() for p in self.params]
        self.n = sum(sizes)
        self.flat = torch.empty(self.n, device=device, dtype=torch.float32)
        self.grad = torch.zeros(self.n, device=device, dtype=torch.float32)
        offs = [0]
        for s in sizes:
            offs.append(offs[-1] + s)
        self.offsets = offs
        for p, a, b in zip(self.params, offs[:-1], offs[1:]):
            self.flat[a:b].copy_(p.detach().reshape(-1).to(device))
            p.data = self.flat[a:b].view(p.shape)
            p.grad = self.grad[a:b].view(p.shape)
        self.seg = torch.tensor(offs, device=device, dtype=torch.int64)

    def zero_grad(self):
        self.grad.zero_()

    def rebind(self, module: nn.Module, flat: torch.Tensor):
        """Point ``module``'s parameters (same layout, e.g. an EMA copy) at ``flat``."""
        ps = list(module.parameters())
        assert len(ps) == len(self.params)
        for p, a, b in zip(ps, self.offsets[:-1], self.offsets[1:]):
            p.data = flat[a:b].view(p.shape)
            p.requires_grad_(False)
