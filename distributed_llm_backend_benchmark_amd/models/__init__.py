"""Model families: the reference's tensor-parallel transformer (1B/7B/13B, forward benchmark)
and GPT-2 (DDP training microbenchmark)."""

from .tp_transformer import LLM, MODEL_CONFIGS, create_model, create_model_from_config

__all__ = ["LLM", "MODEL_CONFIGS", "create_model", "create_model_from_config"]
