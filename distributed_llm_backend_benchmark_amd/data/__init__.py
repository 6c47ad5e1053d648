"""Synthetic data generators (reference ``data_gen.py``)."""

from .synthetic import (SyntheticEmbeddingDataset, SyntheticTokenDataset,
                        create_dataset_from_config)

__all__ = ["SyntheticEmbeddingDataset", "SyntheticTokenDataset", "create_dataset_from_config"]
