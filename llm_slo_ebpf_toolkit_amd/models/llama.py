"""Llama-shaped decoder (random init) -- the instrumented LLM workload of configs 2-4.

REF's demo serves TinyLlama GGUF on CPU through llama.cpp. With no
network there are no weights here, so the workload is a random-init model of a real
architecture (7B Llama shape by default: 32 layers, d=4096, 32 heads, SwiGLU 11008,
RoPE, RMSNorm), bf16 on one MI355X or tensor-parallel over RCCL/xGMI
(``parallel/tensor.py``: column-parallel QKV / gate-up, row-parallel O / down, one
all-reduce after each row-parallel GEMM). TTFT and tokens/s are what the SLO pipeline
measures; token ids are meaningless, the compute and memory traffic are real.

GEMMs go to hipBLASLt through torch.matmul; attention uses PyTorch's fused SDPA (flash
attention on ROCm). The KV cache is preallocated once per (batch, max_seq) in HBM.
"""

from __future__ import annotations

import math
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class LlamaConfig:
    vocab: int = 32000
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 32
    ffn_dim: int = 11008
    max_seq: int = 4096
    rope_theta: float = 10000.0
    norm_eps: float = 1e-5

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    @staticmethod
    def preset(name: str) -> "LlamaConfig":
        if name == "7b":
            return LlamaConfig()
        if name == "8b":  # Llama-3-8B shape (GQA)
            return LlamaConfig(vocab=128256, n_kv_heads=8, ffn_dim=14336, rope_theta=500000.0)
        if name == "1b":  # TinyLlama-1.1B shape (REF demo model)
            return LlamaConfig(vocab=32000, dim=2048, n_layers=22, n_heads=32, n_kv_heads=4, ffn_dim=5632)
        if name == "tiny":  # tests
            return LlamaConfig(vocab=512, dim=256, n_layers=2, n_heads=4, n_kv_heads=2, ffn_dim=688, max_seq=256)
        raise ValueError(f"unknown preset {name!r}")

    def params(self) -> int:
        kv = self.n_kv_heads * self.head_dim
        per_layer = self.dim * (self.dim + 2 * kv) + self.dim * self.dim + 3 * self.dim * self.ffn_dim + 2 * self.dim
        return self.n_layers * per_layer + 2 * self.vocab * self.dim + self.dim


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))
        self.eps = eps

    def forward(self, x):
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)).to(x.dtype) * self.weight


def rope_tables(cfg: LlamaConfig, device, dtype=torch.float32):
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, cfg.head_dim, 2, device=device, dtype=torch.float32) / cfg.head_dim))
    t = torch.arange(cfg.max_seq, device=device, dtype=torch.float32)
    f = torch.outer(t, inv)
    return torch.cos(f).to(dtype), torch.sin(f).to(dtype)


def apply_rope(x, cos, sin):
    """x [B, H, T, D]; cos/sin [T, D/2] (rotate-half convention)."""
    d = x.shape[-1] // 2
    x1, x2 = x[..., :d], x[..., d:]
    c, s = cos[None, None].to(x.dtype), sin[None, None].to(x.dtype)
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig, tp_size: int = 1):
        super().__init__()
        assert cfg.n_heads % tp_size == 0 and cfg.n_kv_heads % tp_size == 0
        self.cfg, self.tp = cfg, tp_size
        self.h = cfg.n_heads // tp_size
        self.kvh = cfg.n_kv_heads // tp_size
        self.hd = cfg.head_dim
        self.wqkv = nn.Linear(cfg.dim, (self.h + 2 * self.kvh) * self.hd, bias=False)  # column-parallel
        self.wo = nn.Linear(self.h * self.hd, cfg.dim, bias=False)                     # row-parallel

    def forward(self, x, cos, sin, cache: Optional[torch.Tensor], pos: int):
        B, T, _ = x.shape
        qkv = self.wqkv(x).view(B, T, self.h + 2 * self.kvh, self.hd).transpose(1, 2)
        q, k, v = qkv.split([self.h, self.kvh, self.kvh], dim=1)
        q = apply_rope(q, cos[pos:pos + T], sin[pos:pos + T])
        k = apply_rope(k, cos[pos:pos + T], sin[pos:pos + T])
        if cache is not None:  # cache [2, B, kvh, max_seq, hd]
            cache[0, :, :, pos:pos + T] = k
            cache[1, :, :, pos:pos + T] = v
            k, v = cache[0, :, :, :pos + T], cache[1, :, :, :pos + T]
        if self.kvh != self.h:
            rep = self.h // self.kvh
            k = k.repeat_interleave(rep, dim=1)
            v = v.repeat_interleave(rep, dim=1)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=(T > 1 and pos == 0))
        return self.wo(o.transpose(1, 2).reshape(B, T, self.h * self.hd))


class MLP(nn.Module):
    def __init__(self, cfg: LlamaConfig, tp_size: int = 1):
        super().__init__()
        assert cfg.ffn_dim % tp_size == 0
        f = cfg.ffn_dim // tp_size
        self.w13 = nn.Linear(cfg.dim, 2 * f, bias=False)  # column-parallel (gate | up)
        self.w2 = nn.Linear(f, cfg.dim, bias=False)       # row-parallel

    def forward(self, x):
        g, u = self.w13(x).chunk(2, dim=-1)
        return self.w2(F.silu(g) * u)


class Block(nn.Module):
    def __init__(self, cfg: LlamaConfig, tp_size: int = 1, reduce=None):
        super().__init__()
        self.attn_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.attn = Attention(cfg, tp_size)
        self.mlp_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.mlp = MLP(cfg, tp_size)
        self.reduce = reduce  # all-reduce after row-parallel GEMMs (tensor parallel)

    def forward(self, x, cos, sin, cache, pos):
        a = self.attn(self.attn_norm(x), cos, sin, cache, pos)
        if self.reduce is not None:
            a = self.reduce(a)
        x = x + a
        m = self.mlp(self.mlp_norm(x))
        if self.reduce is not None:
            m = self.reduce(m)
        return x + m


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig, tp_size: int = 1, reduce=None):
        super().__init__()
        self.cfg = cfg
        self.tp = tp_size
        self.embed = nn.Embedding(cfg.vocab, cfg.dim)
        self.layers = nn.ModuleList(Block(cfg, tp_size, reduce) for _ in range(cfg.n_layers))
        self.norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.lm_head = nn.Linear(cfg.dim, cfg.vocab, bias=False)
        self._rope = None
        self.cache: Optional[torch.Tensor] = None

    @torch.no_grad()
    def random_init(self, seed: int = 0, std: float = 0.02):
        g = torch.Generator(device=self.embed.weight.device).manual_seed(seed)
        for name, p in self.named_parameters():
            if name.endswith("norm.weight") or ".attn_norm." in name or ".mlp_norm." in name:
                p.fill_(1.0)
            else:
                p.normal_(0.0, std, generator=g)
        return self

    def rope(self, device):
        if self._rope is None or self._rope[0].device != device:
            self._rope = rope_tables(self.cfg, device)
        return self._rope

    def alloc_cache(self, batch: int, max_seq: int, dtype, device):
        kvh = self.cfg.n_kv_heads // self.tp
        self.cache = torch.zeros(self.cfg.n_layers, 2, batch, kvh, max_seq, self.cfg.head_dim, dtype=dtype,
                                 device=device)
        return self.cache

    def forward(self, tokens, pos: int = 0):
        cos, sin = self.rope(tokens.device)
        x = self.embed(tokens)
        for i, layer in enumerate(self.layers):
            x = layer(x, cos, sin, None if self.cache is None else self.cache[i], pos)
        return self.lm_head(self.norm(x[:, -1:]))

    @torch.no_grad()
    def generate(self, prompt, max_new: int, on_token=None) -> Dict[str, float]:
        """Greedy decode. Returns TTFT / per-token timings (device-synchronised)."""
        B, T = prompt.shape
        dev = prompt.device
        if self.cache is None or self.cache.shape[2] < B or self.cache.shape[4] < T + max_new:
            self.alloc_cache(B, min(self.cfg.max_seq, T + max_new), self.embed.weight.dtype, dev)
        sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
        sync()
        t0 = time.perf_counter()
        logits = self.forward(prompt, 0)
        nxt = logits.argmax(-1)
        sync()
        ttft = time.perf_counter() - t0
        if on_token:
            on_token(nxt)
        pos = T
        for _ in range(max_new - 1):
            logits = self.forward(nxt, pos)
            nxt = logits.argmax(-1)
            pos += 1
            if on_token:
                on_token(nxt)
        sync()
        total = time.perf_counter() - t0
        dec = max(total - ttft, 1e-9)
        return {"ttft_ms": 1e3 * ttft, "total_ms": 1e3 * total,
                "tokens_per_s": B * (max_new - 1) / dec if max_new > 1 else 0.0, "prompt_tokens": B * T,
                "new_tokens": B * max_new}


def build(preset: str = "7b", device="cuda", dtype=torch.bfloat16, seed: int = 0, tp_size: int = 1,
          reduce=None) -> Llama:
    cfg = LlamaConfig.preset(preset)
    with torch.device(device):
        m = Llama(cfg, tp_size, reduce)
    m = m.to(dtype)
    m.random_init(seed)
    m.eval()
    return m
