"""Serving path of the bundled models: KV-cache generation (``generate.LlamaGenerator``)."""
from .generate import KVCache, LlamaGenerator

__all__ = ["KVCache", "LlamaGenerator"]
