"""utils.mt.data drop-in: TwoStreamBatchSampler (utils/mt/data.py:105-150).

Host-side index logic (no device work).  Each batch is `batch_size -
secondary_batch_size` primary (unlabeled) indices from one permutation of the
primary set, followed by `secondary_batch_size` (labeled) indices from an
endless chain of re-shuffles; len = #primary // primary batch.  The numpy RNG
is consumed in the reference's order (the primary permutation when iteration
starts, each secondary permutation when its first index is needed), so a
seeded run draws the same batches.

For data-parallel training, `shard(rank, world)` returns this rank's sampler
over disjoint index subsets.
"""
import itertools

import numpy as np
from torch.utils.data.sampler import Sampler


class TwoStreamBatchSampler(Sampler):
    def __init__(self, primary_indices, secondary_indices, batch_size, secondary_batch_size):
        self.primary_indices = primary_indices
        self.secondary_indices = secondary_indices
        self.secondary_batch_size = secondary_batch_size
        self.primary_batch_size = batch_size - secondary_batch_size
        assert len(self.primary_indices) >= self.primary_batch_size > 0
        assert len(self.secondary_indices) >= self.secondary_batch_size > 0

    def __iter__(self):
        first = np.random.permutation(self.primary_indices)

        def reshuffles():
            while True:
                yield np.random.permutation(self.secondary_indices)

        prim = iter(first)
        sec = itertools.chain.from_iterable(reshuffles())
        for _ in range(len(self)):
            p = tuple(next(prim) for _ in range(self.primary_batch_size))
            s = tuple(next(sec) for _ in range(self.secondary_batch_size))
            yield p + s

    def __len__(self):
        return len(self.primary_indices) // self.primary_batch_size

    def shard(self, rank, world):
        """Disjoint per-rank index subsets (strided), same per-rank batch shape."""
        return TwoStreamBatchSampler(list(self.primary_indices)[rank::world],
                                     list(self.secondary_indices)[rank::world],
                                     self.primary_batch_size + self.secondary_batch_size,
                                     self.secondary_batch_size)
