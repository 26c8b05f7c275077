"""MI355X-native LLM-SLO observability toolkit.

A from-scratch re-design (not a port) of the capabilities of
``ogulcanaydogan/llm-slo-ebpf-toolkit`` for AMD Instinct MI355X (gfx950):

* ``contracts``   -- SLO-event v1 / incident-attribution v1 / probe-event contracts,
                     compiled JSON-schema validator, semconv keys, toolkit config.
* ``signals``     -- the signal catalogue (9 kernel + 3 derived + 4 GPU signals),
                     capability modes, synthetic generator, metadata enrichers.
* ``collector``   -- record formats, ring-buffer decode, probe manager, pipelines.
* ``correlation`` -- 4-tier span<->signal matching, evaluator, retry-storm detector,
                     multi-signal enrichment (CPU oracle of the GPU join kernel).
* ``models``      -- attribution models: REF-exact naive Bayes, learned Bayes,
                     covariance (LDA) model, rule mapper, metrics.
* ``ops``         -- hand-written HIP/CDNA4 kernels (decode+histogram, LDS-staged
                     correlation join, MFMA posterior/statistics, gate statistics,
                     windowed counts) and their bindings.
* ``runtime``     -- native C++ runtime: pinned MPSC ring, HBM window arena,
                     native replay generator.
* ``pipeline``    -- the per-window GPU engine (streams, overlap, graph capture).
* ``parallel``    -- one-process-per-GPU event-stream data parallelism over RCCL.
* ``evaluation``  -- benchmark bundle, fault replay, release gates, SLO math, prereq.
* ``export``      -- OTLP/HTTP logs, webhooks (generic/PagerDuty/Opsgenie),
                     Prometheus exposition, CD gate.
* ``agent`` / ``cli`` -- the DaemonSet agent and every REF binary.
"""

__version__ = "0.1.0"

PACKAGE_ROOT = __file__.rsplit("/", 1)[0]
