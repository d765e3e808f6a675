"""EPO latent gene pool (evolution.py of the reference, :28-184).

The pool is tiny (num_genes x dim_gene), so selection / crossover / mutation stay on the host in
PyTorch with a private generator per call, seeded from (seed, update, epoch, minibatch) — the
draws are then identical on every rank without a seed all-reduce and reproducible against the
oracle.  The l2-normalised genes are mirrored on the device for the learn step."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def evolve_seed(seed, update, epoch, minibatch):
    return ((int(seed) * 7919 + int(update)) * 7919 + int(epoch)) * 7919 + int(minibatch) & (2 ** 62 - 1)


class LatentGenePool:
    def __init__(self, dim, num_genes_per_island, num_selected, tournament_size, num_elites=1,
                 mutation_std_dev=0.1, num_islands=1, migrate_genes_every=10, num_frac_migrate=0.1, generator=None):
        assert num_islands >= 1 and num_genes_per_island > 2
        assert 2 <= num_selected < num_genes_per_island, 'must select at least 2 genes for mating'
        assert 0. <= num_frac_migrate <= 1.
        self.dim_gene, self.num_islands = dim, num_islands
        self.per, self.num_genes = num_genes_per_island, num_genes_per_island * num_islands
        self.num_selected, self.tournament_size = num_selected, tournament_size
        self.num_children = num_genes_per_island - num_selected
        self.num_elites, self.mutation_std = num_elites, mutation_std_dev
        self.migrate_every, self.frac_migrate = migrate_genes_every, num_frac_migrate
        self.genes = F.normalize(torch.randn(self.num_genes, dim, generator=generator), dim=-1)   # evo.py:63
        self.step = 0

    def __getitem__(self, idx):
        return F.normalize(self.genes[idx], dim=-1)

    @torch.no_grad()
    def evolve_(self, fitnesses, generator=None, temperature=1.5):
        """evo.py:76-184, draws in the reference's order: tournament randn, crossover randn, mutation randn."""
        g = generator
        fit = fitnesses.detach().float().cpu().reshape(self.num_islands, self.per)
        D = self.dim_gene
        genes = self.genes.reshape(self.num_islands, self.per, D)
        sorted_fit, sorted_ids = fit.sort(dim=-1, descending=True)
        sel_ids = sorted_ids[:, :self.num_selected]
        selected = genes.gather(1, sel_ids[..., None].expand(-1, -1, D))
        tourn = torch.randn((self.num_islands, self.num_children, self.num_selected), generator=g).argsort(dim=-1)
        tourn = tourn[..., :self.tournament_size]
        tourn_fit = sorted_fit[..., None].expand(-1, -1, tourn.shape[-1]).gather(1, tourn)
        # the reference indexes the selected genes with tournament *positions* (evo.py:121-127)
        parent_ids = tourn_fit.topk(2, dim=-1).indices.reshape(self.num_islands, -1)
        parents = selected.gather(1, parent_ids[..., None].expand(-1, -1, D))
        parents = parents.reshape(self.num_islands, self.num_children, 2, D).permute(2, 0, 1, 3)
        p1, p2 = parents[0], parents[1]
        children = p1.lerp(p2, (torch.randn(p1.shape, generator=g) / temperature).sigmoid())
        if (self.step + 1) % self.migrate_every == 0 and self.num_islands > 1 and self.frac_migrate > 0.:
            elites = None
            if self.num_elites > 0:
                elites, selected = selected[:, :1], selected[:, 1:]
            k = max(1, int(selected.shape[1] * self.frac_migrate))
            selected, migrants = selected[:, -k:], selected[:, :-k]
            selected = torch.cat((selected, torch.roll(migrants, 1, dims=(1,))), dim=1)
            if elites is not None:
                selected = torch.cat((elites, selected), dim=1)
        out = torch.cat((selected, children), dim=1)
        if self.mutation_std > 0:
            if self.num_elites > 0:
                el, rest = out[:, :1], out[:, 1:]
                rest = rest + torch.randn(rest.shape, generator=g) * self.mutation_std
                out = torch.cat((el, rest), dim=1)
            else:
                out = out + torch.randn(out.shape, generator=g) * self.mutation_std
        self.genes = F.normalize(out.reshape(self.num_genes, D), dim=-1)
        self.step += 1
        return sel_ids
