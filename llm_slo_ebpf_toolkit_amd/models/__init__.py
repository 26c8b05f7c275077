"""L4 attribution models (REF-exact Bayes, learned Bayes, covariance LDA, rule mapper)."""

from .sample import (FaultSample, LABEL_TO_DOMAIN, build_attribution, load_samples_jsonl,  # noqa: F401
                     map_fault_label, write_samples_jsonl)
from .bayes import (LDA, LinearPosteriorModel, NaiveBayes, Posterior, SufficientStats,  # noqa: F401
                    get_model, samples_to_arrays)
from .metrics import (accuracy, build_attributions, confusion_matrix, coverage_accuracy,  # noqa: F401
                      macro_f1, macro_f1_from_confusion, partial_accuracy, per_class_report)
