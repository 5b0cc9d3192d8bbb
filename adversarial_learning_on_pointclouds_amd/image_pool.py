"""Discriminator-input history (the interface of utils/image_pool.py:10-55).

The hot path runs with pool_size=0 (train_classification.py:52 default), where
query() hands its input back unchanged.  With pool_size > 0 the history is one
preallocated device tensor: while it is filling, each queried sample is stored
and returned; once full, each sample is, with probability 1/2, swapped with a
uniformly chosen stored one (the stored one is returned), or else returned as
is.  The draws use Python's `random` module in the same order as the
reference (one random() per sample, one randrange(pool_size) per swap), so a
seeded run makes the same choices.

The draws do not depend on the data, so a query first plans on the host where
each returned row comes from (a batch row, or a slot's content before the
query; a slot swapped twice in one batch hands the second sample the first
one's row) and which batch row each touched slot ends up holding, then applies
the plan as one gather and one scatter on the device instead of a copy per
sample."""
from __future__ import annotations

import random

import torch


class ImagePool:
    def __init__(self, pool_size):
        self.pool_size = int(pool_size)
        self._bank = None  # (pool_size, *sample_shape), allocated on first use
        self._filled = 0

    @property
    def num_imgs(self):
        return self._filled

    def query(self, images):
        if self.pool_size == 0:
            return images
        batch = images.detach()
        shape = (self.pool_size,) + tuple(batch.shape[1:])
        if self._bank is None or (self._filled == 0 and (
                tuple(self._bank.shape) != shape or self._bank.dtype != batch.dtype
                or self._bank.device != batch.device)):
            self._bank = batch.new_empty(shape)  # (re)allocated while the history is empty
        elif (tuple(self._bank.shape) != shape or self._bank.dtype != batch.dtype
              or self._bank.device != batch.device):
            raise ValueError(f"ImagePool: samples of shape {tuple(batch.shape[1:])} {batch.dtype} "
                             f"on {batch.device}, but the history holds "
                             f"{tuple(self._bank.shape[1:])} {self._bank.dtype} on "
                             f"{self._bank.device}")
        n = batch.shape[0]
        src = list(range(n))  # out[i] = rows[src[i]] of cat(batch, bank as it was)
        holds = {}            # slot -> batch row it holds after this query
        for i in range(n):
            if self._filled < self.pool_size:
                holds[self._filled] = i
                self._filled += 1
            elif random.random() > 0.5:
                slot = random.randrange(self.pool_size)
                src[i] = holds.get(slot, n + slot)
                holds[slot] = i
        if all(src[i] == i for i in range(n)):
            out = batch.clone()
        else:
            idx = torch.tensor(src, dtype=torch.int64, device=batch.device)
            out = torch.cat((batch, self._bank)).index_select(0, idx)
        if holds:
            plan = torch.tensor([list(holds), list(holds.values())], dtype=torch.int64,
                                device=batch.device)
            self._bank.index_copy_(0, plan[0], batch.index_select(0, plan[1]))
        return out.requires_grad_(True)
