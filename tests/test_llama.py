"""Random-init Llama workload: shapes, KV-cache decode == full recompute, and tensor
parallel (gloo, 2 ranks) == single-process logits."""

import os
import socket

import pytest
import torch

from llm_slo_ebpf_toolkit_amd.models.llama import Llama, LlamaConfig, build
from llm_slo_ebpf_toolkit_amd.parallel.tensor import build_tp


def test_param_count_7b():
    assert abs(LlamaConfig.preset("7b").params() / 1e9 - 6.74) < 0.05


def test_kv_cache_decode_matches_recompute():
    torch.manual_seed(0)
    m = build("tiny", "cpu", torch.float32)
    prompt = torch.randint(0, m.cfg.vocab, (2, 12))
    out = []
    m.generate(prompt, 5, on_token=out.append)
    toks = torch.cat(out, dim=1)
    # recompute every step without cache
    m.cache = None
    seq = prompt
    for i in range(5):
        nxt = m.forward(seq, 0).argmax(-1)
        assert torch.equal(nxt, toks[:, i:i + 1])
        seq = torch.cat([seq, nxt], dim=1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tp_worker(rank, world, port, path, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.load(path, weights_only=True)
        m = build_tp("tiny", rank, world, "cpu", torch.float32, full_state=full)
        prompt = torch.arange(10).view(1, 10) % m.cfg.vocab
        logits = m.forward(prompt, 0)
        torch.save(logits, f"{out}/r{rank}.pt")
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_tensor_parallel_gloo_matches_single(tmp_path):
    import torch.multiprocessing as mp

    full_model = build("tiny", "cpu", torch.float32, seed=3)
    path = tmp_path / "full.pt"
    torch.save(full_model.state_dict(), path)
    mp.spawn(_tp_worker, args=(2, _free_port(), str(path), str(tmp_path)), nprocs=2, join=True)
    ref = full_model.forward(torch.arange(10).view(1, 10) % full_model.cfg.vocab, 0)
    for r in range(2):
        torch.testing.assert_close(torch.load(tmp_path / f"r{r}.pt", weights_only=True), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_llama_gpu_ttft_small():
    m = build("1b", "cuda")
    prompt = torch.randint(0, m.cfg.vocab, (1, 128), device="cuda")
    r = m.generate(prompt, 8)
    assert r["ttft_ms"] > 0 and r["tokens_per_s"] > 0
