"""Model configurations of the bundled PyTorch-ROCm training chart.

``llama3_8b`` is the headline benchmark model (BASELINE.json config #4); ``gpt2_small`` is config #3
(true GPT-2 architecture: LayerNorm, GELU, learned positions, tied embeddings, biases). The ``tiny_*``
configs are for CPU plumbing tests and GPU smoke runs.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field


@dataclass
class ModelConfig:
    name: str
    arch: str  # "llama" | "gpt2"
    vocab_size: int
    hidden: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    ffn_hidden: int
    max_seq_len: int
    norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    tie_embeddings: bool = False
    init_std: float = 0.02
    extra: dict = field(default_factory=dict)

    @property
    def head_dim(self) -> int:
        return self.hidden // self.n_heads

    def to_dict(self):
        return asdict(self)

    def num_params(self) -> int:
        H, L, V, F = self.hidden, self.n_layers, self.vocab_size, self.ffn_hidden
        D = self.head_dim
        if self.arch == "llama":
            attn = H * (self.n_heads + 2 * self.n_kv_heads) * D + self.n_heads * D * H
            mlp = 3 * H * F
            per = attn + mlp + 2 * H
            emb = V * H * (1 if self.tie_embeddings else 2)
            return L * per + emb + H
        # gpt2
        attn = 3 * H * H + 3 * H + H * H + H
        mlp = 2 * H * F + F + H
        per = attn + mlp + 4 * H
        return L * per + V * H + self.max_seq_len * H + 2 * H

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs per token (fwd + bwd = 3x fwd), matmuls + causal attention."""
        H, L, V = self.hidden, self.n_layers, self.vocab_size
        D = self.head_dim
        if self.arch == "llama":
            mm = L * (H * (self.n_heads + 2 * self.n_kv_heads) * D + self.n_heads * D * H + 3 * H * self.ffn_hidden)
        else:
            mm = L * (4 * H * H + 2 * H * self.ffn_hidden)
        mm += V * H
        attn = L * 2 * self.n_heads * D * seq_len  # QK^T + PV, causal half of 2*2*S*D per head
        return 6.0 * mm + 3.0 * attn


CONFIGS = {
    "llama3_8b": ModelConfig("llama3_8b", "llama", 128256, 4096, 32, 32, 8, 14336, 8192, 1e-5, 500000.0),
    # past one GPU: weights + fp32 AdamW state ~1.1 TB -> tensor parallelism (--tp) inside an 8x MI355X node
    "llama3_70b": ModelConfig("llama3_70b", "llama", 128256, 8192, 80, 64, 8, 28672, 8192, 1e-5, 500000.0),
    "llama3_1b_proxy": ModelConfig("llama3_1b_proxy", "llama", 128256, 2048, 16, 32, 8, 8192, 8192, 1e-5, 500000.0),
    "gpt2_small": ModelConfig("gpt2_small", "gpt2", 50304, 768, 12, 12, 12, 3072, 1024, 1e-5, 0.0,
                              tie_embeddings=True),
    "tiny_llama": ModelConfig("tiny_llama", "llama", 512, 256, 2, 4, 2, 512, 256, 1e-5, 10000.0),
    "tiny_gpt2": ModelConfig("tiny_gpt2", "gpt2", 512, 128, 2, 2, 2, 512, 256, 1e-5, 0.0, tie_embeddings=True),
}


def get_config(name: str, **overrides) -> ModelConfig:
    if name not in CONFIGS:
        raise KeyError(f"unknown model config {name!r}; known: {sorted(CONFIGS)}")
    cfg = CONFIGS[name]
    d = cfg.to_dict()
    d.update(overrides)
    return ModelConfig(**d)
