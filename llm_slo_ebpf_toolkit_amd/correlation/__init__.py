"""L3 correlation: tier matching, multi-signal enrichment, evaluation, retry storms."""

from .match import (DEFAULT_ENRICHMENT_THRESHOLD, DEFAULT_WINDOW_NS, Decision, SignalRef,  # noqa: F401
                    SpanRef, TIERS, enrich_dns, match, within_window)
from .correlator import (Candidate, Correlator, DebugStats, EnrichmentResult, ProcessedBatch,  # noqa: F401
                         SpanRecord, decompose_retrieval)
from .evaluator import (EvalReport, LabeledPair, Prediction, evaluate_gate,  # noqa: F401
                        evaluate_labeled_pairs, load_labeled_pairs)
from .retry_storm import RetryStormDetector  # noqa: F401
