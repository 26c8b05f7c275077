"""Tensor parallelism for the instrumented LLM workload (config 4: TP inference over xGMI).

Megatron-style split of ``models/llama.py``: QKV and gate|up projections are
column-parallel (each rank holds a slice of heads / ffn columns, no communication), O and
down projections are row-parallel and followed by one all-reduce of the [B, T, d]
activations -- two RCCL all-reduces per layer. On MI355X the 8 GPUs of a node are fully
connected by xGMI (7 links x ~153 GB/s per GPU), so decode-step all-reduces are latency
bound (16 KiB at B=1, d=4096, bf16) and prefill ones bandwidth bound on one link per ring
step; TP=8 keeps every shard of a 7B model < 2 GiB, far below 288 GB HBM -- the trade-off
is chosen for TTFT, not capacity.
"""

from __future__ import annotations

from typing import Callable, Optional

import torch

from ..models.llama import Llama, LlamaConfig


def allreduce_fn(group=None) -> Callable[[torch.Tensor], torch.Tensor]:
    import torch.distributed as dist

    def reduce(x: torch.Tensor) -> torch.Tensor:
        dist.all_reduce(x, group=group)
        return x

    return reduce


def _split_qkv(w: torch.Tensor, cfg: LlamaConfig, rank: int, world: int) -> torch.Tensor:
    hd = cfg.head_dim
    q, k, v = w.split([cfg.n_heads * hd, cfg.n_kv_heads * hd, cfg.n_kv_heads * hd], dim=0)
    return torch.cat([q.chunk(world, 0)[rank], k.chunk(world, 0)[rank], v.chunk(world, 0)[rank]], dim=0)


def _split_gate_up(w: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    g, u = w.chunk(2, dim=0)
    return torch.cat([g.chunk(world, 0)[rank], u.chunk(world, 0)[rank]], dim=0)


@torch.no_grad()
def shard_state_dict(full: dict, cfg: LlamaConfig, rank: int, world: int) -> dict:
    """Full-model state dict -> this rank's tensor-parallel shard."""
    out = {}
    for k, v in full.items():
        if k.endswith("attn.wqkv.weight"):
            out[k] = _split_qkv(v, cfg, rank, world).contiguous()
        elif k.endswith("mlp.w13.weight"):
            out[k] = _split_gate_up(v, rank, world).contiguous()
        elif k.endswith("attn.wo.weight") or k.endswith("mlp.w2.weight"):
            out[k] = v.chunk(world, dim=1)[rank].contiguous()
        else:
            out[k] = v
    return out


def build_tp(preset: str, rank: int, world: int, device="cuda", dtype=torch.bfloat16, seed: int = 0,
             group=None, full_state: Optional[dict] = None) -> Llama:
    """This rank's TP shard. With ``full_state`` the shard is cut from it (tests); otherwise
    every rank random-initialises its own slice from a (seed, rank) stream -- the workload
    only needs the right shapes and traffic."""
    cfg = LlamaConfig.preset(preset)
    reduce = allreduce_fn(group) if world > 1 else None
    with torch.device(device):
        m = Llama(cfg, tp_size=world, reduce=reduce)
    m = m.to(dtype)
    if full_state is not None:
        m.load_state_dict(shard_state_dict(full_state, cfg, rank, world))
    else:
        m.random_init(seed * 1000 + rank)
    m.eval()
    return m
