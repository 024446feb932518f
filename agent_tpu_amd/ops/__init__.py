"""Device ops: thin, shape-checked wrappers over the gfx950 HIP kernels.

Every op runs the native kernel for CUDA (ROCm) tensors and a plain PyTorch
reference for CPU tensors; the reference doubles as the numerics oracle in
``tests/kernels``. There is no silent fallback for device tensors: if the
extension cannot load on a GPU, the call raises.
"""
from .linear import linear, fold_rms_into_linear, EPI_BIAS, EPI_GELU, EPI_TANH, EPI_RESIDUAL, EPI_RELU  # noqa: F401
from .linear import linear_ln, fold_ln_into_linear, fold_ok, ln_partials_ref, ln_finalize, row_parts_ref  # noqa: F401
from .linear import row_totals_parts_ref, batch_invariant, set_batch_invariant  # noqa: F401
from .decode import decode_attention, kv_append, gather_rows, beam_topk_rows, beam_reorder_hist, MAX_BANS  # noqa: F401
from .decode import DecEmbed, decode_advance, decode_advance_ok  # noqa: F401
from .decode import beam_select, beam_select_ref, ngram_bans, lm_head_topk, lm_head, LmHead, LM_HEAD_MAX_K  # noqa: F401
from .attention import attention_packed, attention  # noqa: F401
from .qkv_attention import qkv_attention, qkv_attention_ok, qkv_head_order  # noqa: F401
from .norm import layernorm, rmsnorm, embed_layernorm, embed_gather, embed_pos_layernorm  # noqa: F401
from .tokenize import tokenize  # noqa: F401
from .head import classify_head_topk  # noqa: F401
from .reduce import risk_stats, reduce_stats_tensor  # noqa: F401
