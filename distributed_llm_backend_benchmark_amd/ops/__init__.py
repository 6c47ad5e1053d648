"""Python entry points of the gfx950 HIP kernel library (``csrc/`` -> ``_dlbb_hip.so``).

* :mod:`.elementwise` — n-way sum-reduce, cast, strided pack, multi-tensor chunk copy
  (flatten/unflatten/all-to-all packing).
* :mod:`.gemm` — MFMA bf16 GEMM with fused bias / GELU / residual epilogues.
* :mod:`.norm_act` — fused residual+LayerNorm and bias+GELU (fwd + bwd, autograd).
* :mod:`.optim` — flat fused AdamW.
* :mod:`.xent` — fused softmax cross-entropy on bf16 logits; LM-head-fused linear + loss.
* :mod:`.embedding` — token + position embedding, backward accumulating in place (sinks).
* :mod:`._lib` — loader; ``available()``, ``loaded_path()``.
"""

from . import _lib
from ._lib import available, loaded_path, KernelError
from .elementwise import reduce_sum, cast, pack_rows, ChunkTable, ScaleTable, flatten_into
from .gemm import linear
from .norm_act import layernorm, bias_gelu
from .optim import FlatAdamW
from .xent import cross_entropy, linear_cross_entropy
from .attention import causal_attention
from .embedding import embedding

__all__ = ["causal_attention", "available", "loaded_path", "KernelError", "reduce_sum", "cast", "pack_rows",
           "ChunkTable", "ScaleTable", "flatten_into", "linear", "layernorm", "bias_gelu",
           "FlatAdamW", "cross_entropy", "linear_cross_entropy", "embedding"]
