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


def rank_main(rank, world, uq, n_win, q):
    try:
        import numpy as np

        from llm_slo_ebpf_toolkit_amd.ops import load_agent

        # the unique id's bootstrap root lives in the process that made it: rank 0 keeps it
        if rank == 0:
            uid = load_agent().unique_id()
            for _ in range(world - 1):
                uq.put(uid)
        else:
            uid = uq.get(timeout=120)

        from llm_slo_ebpf_toolkit_amd.collector.records import framed_rows
        from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator
        from llm_slo_ebpf_toolkit_amd.pipeline.window import Cut, RingWindowSource, WindowPipeline, build_replay_images
        from llm_slo_ebpf_toolkit_amd.runtime import load

        cfg = ReplayConfig(scenario="full", events_per_window=1 << 16, spans_per_window=2048, n_services=16, seed=11,
                           shard=rank)
        gen = ReplayGenerator(cfg)
        wins = [gen.next_window() for _ in range(n_win)]
        imgs = build_replay_images(wins, user_rec=24)
        sig_cap = max(framed_rows(i.framed) + len(i.user) for i in imgs)
        user_cap = 1 << int(np.ceil(np.log2(max(len(i.user) for i in imgs))))
        xchg = 4096
        import torch

        dev = rank % max(1, torch.cuda.device_count())  # one GPU per rank where there are enough
        pipe = WindowPipeline(sig_cap, 2048, 16, dev, (uid, rank, world), model="bayes_learned",
                              user_cap=min(user_cap, sig_cap), import_cap=(world - 1) * xchg, xchg_cap=xchg)
        pods = np.unique(np.concatenate([w.events["pod_id"] for w in wins]))
        sn = {}
        for w in wins:
            v = (w.events["svc_id"].astype(np.uint32) << np.uint32(16)) | w.events["node_id"].astype(np.uint32)
            sn.update(zip(w.events["pod_id"].tolist(), v.tolist()))
        pipe.eng.set_pods(pods.astype(np.uint32), np.array([sn[p] for p in pods.tolist()], dtype=np.uint32))
        rt = load()
        rb = rt.Ringbuf.create_shm(f"/mislo-rpp-{os.getpid()}", 1 << 24)
        user, spans = rt.HostRing(1 << 16, 24), rt.HostRing(1 << 14, 64)
        src = RingWindowSource(pipe, rb, user, spans)
        groups, own, gathered = 0, [], []
        for i, img in enumerate(imgs):
            assert rb.append_framed(img.framed)
            user.push(img.user)
            spans.push(img.spans)
            k = src.stage(Cut(rb.producer_pos, user.head, spans.head, img.bases), img.n_groups, img.labels)["k"]
            groups += img.n_groups
            res = pipe.results(k, img.n_groups)
            own.append(np.asarray(res["pred"]).tolist())
            gathered.append([np.asarray(r["pred"]).tolist() for r in pipe.results_all(k, img.n_groups)])
        src.drain()
        summ = pipe.summary()
        q.put({"rank": rank, "ok": True, "groups": groups, "confusion_sum": int(np.asarray(summ["confusion"]).sum()),
               "hist_sum": float(np.asarray(summ["hist"]).sum()),
               "import_state": [int(x) for x in pipe.eng.import_state()], "own": own, "gathered": gathered})
        pipe.eng.close()
    except Exception as exc:  # reported to the parent; RCCL refusals included
        q.put({"rank": rank, "ok": False, "error": f"{type(exc).__name__}: {exc}", "tb": traceback.format_exc()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=4)
    ap.add_argument("--wait", type=float, default=90.0, help="seconds to wait for each rank")
    a = ap.parse_args()
    world = 2
    ctx = mp.get_context("spawn")  # no GPU state in the parent: each rank initialises its own
    uq, q = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=rank_main, args=(r, world, uq, a.windows, q), daemon=True) for r in range(world)]
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
    r0, r1 = out[0], out[1]
    checks = {
        "totals_identical": r0["hist_sum"] == r1["hist_sum"] and r0["confusion_sum"] == r1["confusion_sum"],
        "confusion_counts_both_shards": r0["confusion_sum"] == r0["groups"] + r1["groups"],
        "gather_slices_match": all(g[0] == r0["own"][i] and g[1] == r1["own"][i]
                                   for i, g in enumerate(r0["gathered"])),
        "imports_seen": [r0["import_state"][:2], r1["import_state"][:2]],
    }
    ok = checks["totals_identical"] and checks["confusion_counts_both_shards"] and checks["gather_slices_match"]
    print(json.dumps({"result": "ok" if ok else "mismatch", "checks": checks,
                      "groups": [r0["groups"], r1["groups"]], "confusion_sum": r0["confusion_sum"]}))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
