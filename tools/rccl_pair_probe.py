"""Two-rank RCCL probe of the window engine's data plane.

Rank r places its engine on device r mod #GPUs and the two build one RCCL communicator (the
engine's own, ``WindowEngine::init_comm``). Each rank runs its node shard of the same replay windows through
the BPF-ring path with the in-window trace-row all-gather enabled, then checks what RCCL
delivered:
* the packet all-reduce: both ranks hold identical node-wide totals, and the confusion matrix
  counts every incident of both shards;
* the incident all-gather: rank r's slice of the gathered results equals rank r's own results.
On a one-GPU box RCCL refuses two ranks on one device (``ncclInvalidUsage``, measured:
profiles/r2_rccl_pair_one_gpu.log); the probe then reports that and exits 3. The multi-GPU scaling run itself belongs to
the driver (bench.py under torch.distributed.run).

usage: python tools/rccl_pair_probe.py [--windows 4]
"""

import argparse
import json
import multiprocessing as mp
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_windows(pipe, imgs, pods_sn, tag):
    """The windows through one pipeline's BPF-ring path: per window the node-wide packet, this
    rank's incident results and the all-gathered results of every rank."""
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.pipeline.window import Cut, RingWindowSource
    from llm_slo_ebpf_toolkit_amd.runtime import load

    pipe.eng.set_pods(*pods_sn)
    rt = load()
    rb = rt.Ringbuf.create_shm(f"/mislo-rpp-{os.getpid()}-{tag}", 1 << 24)
    user, spans = rt.HostRing(1 << 16, 24), rt.HostRing(1 << 14, 64)
    src = RingWindowSource(pipe, rb, user, spans)
    out = []
    for img in imgs:
        assert rb.append_framed(img.framed)
        user.push(img.user)
        spans.push(img.spans)
        k = src.stage(Cut(rb.producer_pos, user.head, spans.head, img.bases), img.n_groups, img.labels)["k"]
        pipe.wait(k)
        res = pipe.results(k, img.n_groups)
        out.append({"packet": np.asarray(pipe.packet(k)["hist"]).astype(np.int64).tolist(),
                    "confusion": np.asarray(pipe.packet(k)["confusion"]).astype(np.int64).tolist(),
                    "feat": np.asarray(res["feat"]).tolist(), "post": np.asarray(res["post"]).tolist(),
                    "pred": np.asarray(res["pred"]).tolist(),
                    "gathered": [np.asarray(r["pred"]).tolist() for r in pipe.results_all(k, img.n_groups)]})
    src.drain()
    return out, [int(x) for x in pipe.eng.import_state()] if hasattr(pipe.eng, "import_state") else []


def rank_main(rank, world, uq, n_win, q, port, engine):
    """Rank ``rank``: its node shard of the replay windows through the GPU engine (RCCL over xGMI:
    packet all-reduce, incident all-gather, in-window trace-row all-gather), then the same windows
    through the CPU engine (the oracle of every kernel, pipeline/cpu.py) over gloo -- the same
    protocol with host collectives. ``engine`` = cpu runs the oracle twice (a rehearsal of this
    probe on a host without GPUs)."""
    try:
        import numpy as np

        from llm_slo_ebpf_toolkit_amd.collector.records import framed_rows
        from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator
        from llm_slo_ebpf_toolkit_amd.pipeline.window import WindowPipeline, build_replay_images

        cfg = ReplayConfig(scenario="full", events_per_window=1 << 16, spans_per_window=2048, n_services=16, seed=11,
                           shard=rank)
        gen = ReplayGenerator(cfg)
        wins = [gen.next_window() for _ in range(n_win)]
        imgs = build_replay_images(wins, user_rec=24)
        sig_cap = max(framed_rows(i.framed) + len(i.user) for i in imgs)
        user_cap = 1 << int(np.ceil(np.log2(max(len(i.user) for i in imgs))))
        xchg = 4096
        pods = np.unique(np.concatenate([w.events["pod_id"] for w in wins]))
        sn = {}
        for w in wins:
            v = (w.events["svc_id"].astype(np.uint32) << np.uint32(16)) | w.events["node_id"].astype(np.uint32)
            sn.update(zip(w.events["pod_id"].tolist(), v.tolist()))
        pods_sn = (pods.astype(np.uint32), np.array([sn[p] for p in pods.tolist()], dtype=np.uint32))
        kw = dict(model="bayes", learn=False, user_cap=min(user_cap, sig_cap), import_cap=(world - 1) * xchg,
                  xchg_cap=xchg)
        import torch.distributed as dist

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        if engine == "gpu":
            from llm_slo_ebpf_toolkit_amd.ops import load_agent

            # the unique id's bootstrap root lives in the process that made it: rank 0 keeps it
            if rank == 0:
                uid = load_agent().unique_id()
                for _ in range(world - 1):
                    uq.put(uid)
            else:
                uid = uq.get(timeout=120)
            import torch

            dev = rank % max(1, torch.cuda.device_count())  # one GPU per rank where there are enough
            pipe = WindowPipeline(sig_cap, 2048, 16, dev, (uid, rank, world), **kw)
        else:
            pipe = WindowPipeline(sig_cap, 2048, 16, engine="cpu", group=dist.group.WORLD, **kw)
        dev_out, imports = run_windows(pipe, imgs, pods_sn, "dev")
        pipe.eng.close()
        cpu = WindowPipeline(sig_cap, 2048, 16, engine="cpu", group=dist.group.WORLD, **kw)
        ref_out, _ = run_windows(cpu, imgs, pods_sn, "cpu")
        groups = sum(i.n_groups for i in imgs)
        q.put({"rank": rank, "ok": True, "groups": groups, "dev": dev_out, "ref": ref_out, "import_state": imports})
        dist.destroy_process_group()
    except Exception as exc:  # reported to the parent; RCCL refusals included
        q.put({"rank": rank, "ok": False, "error": f"{type(exc).__name__}: {exc}", "tb": traceback.format_exc()})


def compare(out) -> dict:
    """Each rank's device windows against the CPU oracle's, and the RCCL-specific properties."""
    import numpy as np

    checks = {"packets_equal_oracle": True, "features_equal_oracle": True, "posteriors_close": True,
              "predictions_equal_oracle": True, "gathered_equal_oracle": True, "totals_identical_across_ranks": True,
              "gather_slices_match": True}
    r0, r1 = out[0], out[1]
    for r in (r0, r1):
        for d, c in zip(r["dev"], r["ref"]):
            checks["packets_equal_oracle"] &= d["packet"] == c["packet"] and d["confusion"] == c["confusion"]
            checks["features_equal_oracle"] &= d["feat"] == c["feat"]
            checks["posteriors_close"] &= bool(np.allclose(np.asarray(d["post"])[:, :10], np.asarray(c["post"])[:, :10],
                                                           rtol=1e-9, atol=1e-12))
            checks["predictions_equal_oracle"] &= d["pred"] == c["pred"]
            checks["gathered_equal_oracle"] &= d["gathered"] == c["gathered"]
    for a, b in zip(r0["dev"], r1["dev"]):  # the all-reduce gives both ranks the node-wide packet
        checks["totals_identical_across_ranks"] &= a["packet"] == b["packet"] and a["confusion"] == b["confusion"]
    for i, d in enumerate(r0["dev"]):  # rank r's slice of the all-gather is rank r's own results
        checks["gather_slices_match"] &= d["gathered"][0] == r0["dev"][i]["pred"] and d["gathered"][1] == r1["dev"][i]["pred"]
    checks["confusion_counts_both_shards"] = int(np.asarray(r0["dev"][-1]["confusion"]).sum()) > 0
    return checks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=4)
    ap.add_argument("--wait", type=float, default=90.0, help="seconds to wait for each rank")
    ap.add_argument("--engine", default="gpu", choices=("gpu", "cpu"),
                    help="cpu: both passes on the CPU engine (a rehearsal of the probe without GPUs)")
    a = ap.parse_args()
    world = 2
    import socket

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")  # no GPU state in the parent: each rank initialises its own
    uq, q = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=rank_main, args=(r, world, uq, a.windows, q, port, a.engine), daemon=True)
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        m = q.get(timeout=a.wait)
        out[m["rank"]] = m
    for p in procs:
        p.join(60)
    errs = [m for m in out.values() if not m["ok"]]
    if errs:
        print(json.dumps({"result": "rccl_refused_or_failed", "errors": [e["error"] for e in errs]}))
        for e in errs:
            print(e["tb"], file=sys.stderr)
        sys.exit(3)
    checks = compare(out)
    ok = all(v for k, v in checks.items())
    print(json.dumps({"result": "ok" if ok else "mismatch", "checks": checks,
                      "groups": [out[0]["groups"], out[1]["groups"]],
                      "imports_seen": [out[0]["import_state"][:2], out[1]["import_state"][:2]]}))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
