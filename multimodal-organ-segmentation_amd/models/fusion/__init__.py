"""Fusion modules (mirror of the reference's src/models/fusion/).  Only the
cross-attention modules are on the engine: the reference never instantiates
any of these from build_model, so they are module-level
drop-ins."""
from .attention_fusion import BidirectionalCrossAttention, CrossAttentionFusion

__all__ = ["CrossAttentionFusion", "BidirectionalCrossAttention"]
