"""Synthetic inputs (no datasets / checkpoints are available or needed).

* :class:`SyntheticEmbeddingDataset` — reference ``data_gen.py:10-53``: ONE fixed bf16
  ``[B, S, H]`` tensor seeded with ``input.seed`` and returned on every call, identical on all
  ranks (replicated TP input). Generated directly in device memory (the reference builds it on
  the CPU, ``data_gen.py:38-44``).
* :class:`SyntheticTokenDataset` — token batches for the GPT-2 DDP microbenchmark: a fixed pool
  of random token ids per rank (rank-offset seed, so DP ranks see different data), cycled.
"""

from __future__ import annotations

from typing import Dict, Tuple

import torch


class SyntheticEmbeddingDataset:
    def __init__(self, batch_size: int, sequence_length: int, hidden_size: int, seed: int = 42,
                 device: torch.device = torch.device("cpu"), dtype=torch.bfloat16):
        self.batch_size, self.sequence_length, self.hidden_size = batch_size, sequence_length, hidden_size
        self.seed = seed
        g = torch.Generator(device=device)
        g.manual_seed(seed)
        self.fixed_batch = torch.randn(batch_size, sequence_length, hidden_size, generator=g,
                                       device=device, dtype=torch.float32).to(dtype)

    def get_batch(self) -> torch.Tensor:
        return self.fixed_batch


def create_dataset_from_config(config: Dict, device: torch.device) -> SyntheticEmbeddingDataset:
    """Reference ``data_gen.py:56-73``."""
    return SyntheticEmbeddingDataset(
        batch_size=int(config["input"]["batch_size"]),
        sequence_length=int(config["input"]["sequence_length"]),
        hidden_size=int(config["model"]["hidden_size"]),
        seed=int(config["input"]["seed"]),
        device=device)


class SyntheticTokenDataset:
    def __init__(self, batch_size: int, seq_len: int, vocab_size: int, rank: int = 0,
                 seed: int = 1337, pool: int = 4, device: torch.device = torch.device("cpu")):
        g = torch.Generator(device=device)
        g.manual_seed(seed + 7919 * rank)
        self.data = torch.randint(0, vocab_size, (pool, batch_size, seq_len + 1), generator=g,
                                  device=device, dtype=torch.int64)
        self.i = 0

    def get_batch(self) -> Tuple[torch.Tensor, torch.Tensor]:
        b = self.data[self.i % self.data.shape[0]]
        self.i += 1
        return b[:, :-1], b[:, 1:]
